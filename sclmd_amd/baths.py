"""Bath models with sclmd's API (sclmd/baths.py): ebath (time-local electron bath with bias terms)
and phbath (phonon bath with a memory kernel).

The bath objects hold parameters, the friction kernel and the noise factorisation.  Their forces
(bforce, baths.py:224-255 / 448-458) are evaluated inside the HIP stepper, not here.
Deviation: invalid shapes raise ValueError instead of print + sys.exit (baths.py:115-116, ...).
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import noise as _noise
from . import units as U
from .functions import antisymmetrize, chkShape, flinterp_many, interp_weights, symmetrize


def exlist(a, indices):
    """The rows of a at the given indices (baths.py:12-14)."""
    return np.asarray(a)[indices]


def gamt(tl, wl, gwl, gam, eta_ad=0):
    """Friction kernel in time, K(t) = (2 wl[-1]/pi) mean_w Gamma(w) cos(w t) (baths.py:19-52),
    evaluated as one matrix product cos(w t) . Gamma(w) over all times and frequencies."""
    tl = np.asarray(tl, dtype=float)
    wl = np.asarray(wl, dtype=float)
    g = flinterp_many(wl, gwl, gam)            # (nw, nc, nc)
    shape = g.shape[1:]
    g2 = g.reshape(len(wl), -1)
    nw = len(wl)
    if eta_ad == 0:
        c = np.cos(np.outer(tl, wl))
        k = (c @ g2) * (2.0 * wl[-1] / np.pi / nw)
    else:
        w = wl[None, :]
        tt = tl[:, None]
        c = (w / (w - 1j * eta_ad) * np.exp(-1j * w * tt - eta_ad * tt)
             + w / (w + 1j * eta_ad) * np.exp(1j * w * tt - eta_ad * tt))
        k = (np.real(c) @ g2) * (wl[-1] / np.pi / nw)
    return np.real(k).reshape((len(tl),) + shape)


def gmem_coefficients(tl, wl, gwl, eta_ad=0):
    """W (len(tl), len(gwl)) with gamt(tl, wl, gwl, gam, eta_ad) == W . gam (baths.py:19-52).

    flinterp (functions.py:117-134) is linear in the spectrum -- two weights per frequency -- so
    the reference's (t, w) double loop factors into scale * C(t, w) . I(w -> gwl): the device
    builds the kernel as ONE contraction over the ngw spectrum nodes (gle_add_bath_gmem)."""
    tl = np.asarray(tl, dtype=float)
    wl = np.asarray(wl, dtype=float)
    gwl = np.asarray(gwl, dtype=float)
    nw = len(wl)
    interp = np.zeros((nw, len(gwl)))
    for k, x in enumerate(wl):
        i, j, wi, wj = interp_weights(x, gwl)
        interp[k, i] += wi
        interp[k, j] += wj
    if eta_ad == 0:
        c = np.cos(np.outer(tl, wl)) * (2.0 * wl[-1] / np.pi / nw)
    else:
        w = wl[None, :]
        tt = tl[:, None]
        c = np.real(w / (w - 1j * eta_ad) * np.exp(-1j * w * tt - eta_ad * tt)
                    + w / (w + 1j * eta_ad) * np.exp(1j * w * tt - eta_ad * tt)) * (wl[-1] / np.pi / nw)
    return c @ interp


def _eigh_parts(spec):
    """(evals, evecs) of a stack of matrices, split over threads with one BLAS thread each (numpy
    releases the GIL): every matrix goes through the same single-threaded LAPACK call however the
    stack is split (across threads, or across the ranks of a node: noise.NodeShare.gather)."""
    n = spec.shape[0]
    if n == 0:
        return np.zeros((0, spec.shape[1])), np.zeros(spec.shape, dtype=spec.dtype)
    nthr = max(1, min(16, os.cpu_count() or 1, n))
    parts = np.array_split(np.arange(n), min(n, 4 * nthr))
    try:
        from threadpoolctl import threadpool_limits
        lim = threadpool_limits(1)
    except Exception:  # pragma: no cover
        lim = None
    try:
        with ThreadPoolExecutor(nthr) as ex:
            res = list(ex.map(lambda ix: np.linalg.eigh(spec[ix]), parts))
    finally:
        if lim is not None:
            lim.restore_original_limits()
    return np.concatenate([r[0] for r in res]), np.concatenate([r[1] for r in res])


def _factor_from(ev, vec):
    f = _noise.NoiseFactor.__new__(_noise.NoiseFactor)
    f.nfreq, f.nc = vec.shape[0], vec.shape[1]
    f.evals = ev
    f.evecs = vec
    f.pos = f.evals > 0
    f.sigma = np.sqrt(np.where(f.pos, f.evals, 0.0))
    f.complex = np.iscomplexobj(f.evecs)
    return f


def _eigh_stack(spec):
    """eigh of a stack of matrices; large stacks are split over threads (numpy releases the GIL)."""
    n = spec.shape[0]
    if spec.shape[-1] < 64 or n < 64:
        return _noise.NoiseFactor(spec)
    nthr = min(16, os.cpu_count() or 1)
    parts = np.array_split(np.arange(n), 4 * nthr)
    try:
        from threadpoolctl import threadpool_limits
        lim = threadpool_limits(1)   # one BLAS thread per worker: no oversubscription
    except Exception:  # pragma: no cover
        lim = None
    try:
        with ThreadPoolExecutor(nthr) as ex:
            res = list(ex.map(lambda ix: np.linalg.eigh(spec[ix]), parts))
    finally:
        if lim is not None:
            lim.restore_original_limits()
    f = _noise.NoiseFactor.__new__(_noise.NoiseFactor)
    f.nfreq, f.nc = n, spec.shape[1]
    f.evals = np.concatenate([r[0] for r in res])
    f.evecs = np.concatenate([r[1] for r in res])
    f.pos = f.evals > 0
    f.sigma = np.sqrt(np.where(f.pos, f.evals, 0.0))
    f.complex = np.iscomplexobj(f.evecs)
    return f


def _digest(*arrays):
    """Content fingerprint of the arrays a noise spectrum is built from (xxh3 over shape, dtype and
    bytes): an array edited in place, or replaced by one that reuses a freed array's id(), changes
    the key, so cached noise factors are never reused for a different spectrum."""
    import xxhash

    h = xxhash.xxh3_64()
    for a in arrays:
        if a is None:
            h.update(b"none")
            continue
        a = np.ascontiguousarray(np.asarray(a))
        h.update(repr((a.shape, a.dtype.str)).encode())
        h.update(a.view(np.uint8).reshape(-1).data)
    return h.hexdigest()


class _BathBase:
    kind = None

    def _noise_key(self):
        raise NotImplementedError

    def bforce(self, t, phis, qhis):
        """bath.bforce (baths.py:224-255 / 448-458) is evaluated inside the HIP stepper as part of
        md.force (no host copy of the per-step force exists): raises."""
        raise NotImplementedError("%s.bforce runs on the device inside md.force / the stepper (gle_run, "
                                  "gle_step_begin / gle_step_end); there is no host evaluation" % type(self).__name__)

    def noise_factor(self, share=None):
        """Eigendecomposition of the noise spectrum, cached until a parameter changes.  share: a
        noise.NodeShare -- the node's ranks each decompose a block of the frequencies and exchange
        the blocks, the same factor bit for bit as one rank's _eigh_parts."""
        key = self._noise_key()
        if getattr(self, "_fac_key", None) != key:
            spec = self._spectrum()
            n, nc = spec.shape[0], spec.shape[1]
            # frequencies whose matrix is exactly zero (above the cutoff: most of them) are not
            # decomposed: eigenvalues 0 with unit eigenvectors, no vargau draw (noise.py:297-303) and a
            # zero factor, what LAPACK returns for them (C3: 99 of 2049 frequencies are nonzero)
            nz = np.flatnonzero(spec.reshape(n, -1).any(axis=1))
            if share is not None and share.world > 1 and len(nz) >= 2 * share.world:
                import hashlib

                tag = "f%s" % hashlib.sha1(repr(key).encode()).hexdigest()[:16]
                ev_nz, vec_nz = share.gather(tag, len(nz), lambda lo, hi: _eigh_parts(spec[nz[lo:hi]]))
            else:
                ev_nz, vec_nz = _eigh_parts(spec[nz])
            ev = np.zeros((n, nc))
            vec = np.zeros(spec.shape, dtype=np.result_type(spec.dtype, vec_nz.dtype))
            vec[:] = np.eye(nc)
            ev[nz] = ev_nz
            vec[nz] = vec_nz
            self._fac = _factor_from(ev, vec)
            self._fac_key = key
        return self._fac

    @property
    def noise(self):
        src = getattr(self, "_noise_src", None)
        if src is not None:  # realisation lives on the device of an md object
            stepper, bid = src
            n = stepper.get_noise(bid)
            return n[0] if n.shape[0] == 1 else n
        return self._noise_host

    @noise.setter
    def noise(self, value):
        self._noise_host = None if value is None else np.asarray(value, dtype=float)
        self._noise_src = None
        self._noise_version = getattr(self, "_noise_version", 0) + 1

    def gnoi(self):
        """Generate one realisation with the global numpy RNG (reference draw order) on the device."""
        if self.nmd is None or self.dt is None:
            raise ValueError("%s.gnoi: dt and nmd must be set" % type(self).__name__)
        self.noise = _noise.generate(self.noise_factor(), self.dt, self.nmd)[0]

    def SetMDsteps(self, dt, nmd):
        self.dt, self.nmd = dt, nmd
        self.cur = np.zeros(nmd)


class ebath(_BathBase):
    """Electron bath (baths.py:55-255).  cats are DOF indices (baths.py:80)."""

    kind = "ebath"

    def __init__(self, cats, T, dt, nmd, wmax=None, nw=None, bias=0., efric=None, exim=None,
                 exip=None, zeta1=None, zeta2=None, classical=False, zpmotion=True):
        self.cats = np.array(cats, dtype=int)
        self.cids = np.array(cats, dtype=int)
        self.nc = len(self.cids)
        self.T, self.wmax = T, wmax
        self.nw, self.bias = nw, bias
        self.dt, self.nmd = dt, nmd
        self.cur = np.zeros(nmd)
        self.classical = classical
        self.zpmotion = zpmotion
        self.wl = None if (nw is None or wmax is None) else [self.wmax * i / nw for i in range(nw)]
        self.CheckEmat(efric, exim, exip, zeta1, zeta2)
        self.ml = 1
        self.noise = None

    def CheckEmat(self, efric=None, exim=None, exip=None, zeta1=None, zeta2=None):
        """Symmetrise efric/exip/zeta1, antisymmetrise exim/zeta2 (baths.py:100-174)."""
        if efric is None:
            self.efric = self.kernel = self.exim = self.exip = self.zeta1 = self.zeta2 = None
            self.ebath = False
            return
        n = chkShape(efric)
        if n != self.nc:
            raise ValueError("ebath.CheckEmat: efric shape error")
        self.efric = symmetrize(efric)
        self.kernel = np.array([self.efric])
        z = np.zeros((n, n))
        self.exip, self.exim, self.zeta1, self.zeta2 = z.copy(), z.copy(), z.copy(), z.copy()
        self.ebath = True
        for name, m, op in (("exim", exim, antisymmetrize), ("exip", exip, symmetrize),
                            ("zeta1", zeta1, symmetrize), ("zeta2", zeta2, antisymmetrize)):
            if m is not None:
                if chkShape(m) != self.nc:
                    raise ValueError("ebath.CheckEmat: the dimension of %s is wrong" % name)
                setattr(self, name, op(m))

    def GetSig(self):
        """Effective retarded self-energy in the wide-band limit on the frequencies wl
        (baths.py:194-208): sig(w) = -i w (efric + bias zeta2) + bias zeta1 - bias exim."""
        if self.wl is None:
            raise ValueError("ebath.GetSig: wl is not set")
        z = np.zeros((self.nc, self.nc))
        e = lambda m: z if m is None else np.asarray(m)  # noqa: E731
        v = float(self.bias)
        self.sig = np.array([-1j * w * (e(self.efric) + v * e(self.zeta2)) + v * e(self.zeta1) - v * e(self.exim)
                             for w in self.wl], dtype=complex).reshape(len(self.wl), self.nc, self.nc)
        return self.sig

    def setbias(self, bias=0.0):
        self.bias = bias

    def biased(self):
        """Bias friction terms are active only if exim, zeta1, zeta2 are all nonzero (baths.py:233)."""
        return bool(self.exim.any() and self.zeta1.any() and self.zeta2.any())

    def _noise_key(self):
        return ("e", self.T, self.bias, self.wmax, self.dt, self.nmd, self.classical, self.zpmotion,
                _digest(self.efric, self.exim, self.exip))

    def _spectrum(self):
        if not self.ebath:
            raise ValueError("ebath.gnoi: ebath is False (no efric)")
        return _noise.electron_spectrum(self.efric, self.exim, self.exip, self.bias, self.T, self.wmax,
                                        self.dt, self.nmd, self.classical, self.zpmotion)

    # streamed factors (noise.stream_factor_chunks): A(w) = aw (efric - exip) + awm/2 (exip + i exim)
    # + awp/2 (exip - i exim), hermitianised (noise.py:171-186), with aw, awm, awp >= 0
    def _shared_matrices(self):
        from .functions import hermitianize

        e = np.asarray(self.efric, dtype=float)
        x = np.asarray(self.exip, dtype=float)
        y = np.asarray(self.exim, dtype=float)
        return [("0", hermitianize((e - x).astype(complex))), ("m", hermitianize(0.5 * (x + 1j * y))),
                ("p", hermitianize(0.5 * (x - 1j * y)))]

    def _spectrum_term(self, i, matrix=True):
        """(kind, shared key, scale, dense matrix or None) of frequency i; matrix=False classifies
        without building the dense matrix."""
        dw = 2.0 * np.pi / self.dt / self.nmd
        delta = self.dt * self.nmd
        w = dw * i
        c = np.array([delta * _noise.equ(w, self.wmax, self.T, self.classical, self.zpmotion),
                      delta * _noise.equ(U.hbar * w - self.bias, self.wmax, self.T, self.classical, self.zpmotion),
                      delta * _noise.equ(U.hbar * w + self.bias, self.wmax, self.T, self.classical, self.zpmotion)])
        nz = np.flatnonzero(c)
        if len(nz) == 0:
            return "zero", None, 0.0, None
        if len(nz) == 1:
            return "shared", "0mp"[nz[0]], float(c[nz[0]]), None
        if not matrix:
            return "dense", None, 1.0, None
        m = c[0] * self.efric
        m = m + (-0.5 * c[0] * self.exip + 0.5 * c[1] * (self.exip + 1j * self.exim))
        m = m + (-0.5 * c[0] * self.exip + 0.5 * c[2] * (self.exip - 1j * self.exim))
        from .functions import hermitianize

        return "dense", None, 1.0, hermitianize(m)


class phbath(_BathBase):
    """Phonon bath (baths.py:258-458)."""

    kind = "phbath"

    def __init__(self, T, cats, debye, nw, dt, nmd, ml=None, mcof=2.0, sig=None, gamma=None, gwl=None,
                 K00=None, K01=None, V01=None, eta_ad=0, classical=False, zpmotion=True):
        self.classical = classical
        self.zpmotion = zpmotion
        self.T, self.debye, self.cats = T, debye, np.array(cats, dtype=int)
        self.K00, self.K01, self.V01 = K00, K01, V01
        self.dt, self.nmd, self.ml = dt, nmd, ml
        self.kernel = None
        self.cids = np.array(cats, dtype=int)
        self.nc = len(self.cids)
        self.wmax = mcof * debye
        self.local = False
        self.nw = nw
        self.wl = [self.wmax * i / nw for i in range(nw)]
        self.gamma = gamma
        self.sig = sig
        self.gwl = gwl
        self.cur = np.zeros(nmd)
        self.eta_ad = eta_ad
        self.noise = None
        if self.UseK():
            raise NotImplementedError("phbath: self-energy from K00/K01/V01 is not implemented "
                                      "(the reference exits here too, baths.py:316-320)")
        elif self.UseG() or self.UsePi():
            if self.UsePi():
                if len(self.sig[0]) != self.nc:
                    raise ValueError("phbath: inconsistent cids and sig")
                self.ggamma()
            if len(self.gamma[0]) != self.nc:
                raise ValueError("phbath: inconsistent cids and gamma")
        else:
            # Debye model, time-local friction (baths.py:333-340)
            self.gamma = np.array([np.diag(debye * np.pi / 6.0 + np.zeros(int(self.nc)))])
            self.gwl = np.array([0])
            self.local = True
            self.ml = 1

    def SetMemlen(self, len):
        self.ml = len

    def SetT(self, T):
        self.T = T

    def UseG(self):
        return self.gamma is not None and self.gwl is not None

    def UsePi(self):
        return self.sig is not None and self.gwl is not None

    def UseK(self):
        return self.K00 is not None and self.K01 is not None and self.V01 is not None

    def ggamma(self):
        """Gamma(w) = -Im Sigma(w) / w, w = 0 taking the next point's value (baths.py:375-395)."""
        sig, wl = np.asarray(self.sig), self.gwl
        a = []
        for i in range(len(wl)):
            j = i + 1 if wl[i] == 0 else i
            a.append(-np.imag(sig[j]) / wl[j])
        self.gamma = np.array(a)

    @property
    def kernel(self):
        """The memory kernel [ml][nc][nc].  After gmem(on_device=True) it is built on the device
        when the bath is added to an md object; reading it here evaluates the same contraction
        W . gamma on the host (once)."""
        k = self.__dict__.get("_kernel")
        rec = self.__dict__.get("_gmem")
        if k is None and rec is not None:
            W, G = rec
            k = (W @ np.asarray(G).reshape(len(G), -1)).reshape((W.shape[0],) + np.shape(G)[1:])
            self.__dict__["_kernel"] = k
        return k

    @kernel.setter
    def kernel(self, value):
        self.__dict__["_kernel"] = value
        self.__dict__["_gmem"] = None

    @property
    def gmem_recipe(self):
        """(W, gamma) of a device-built kernel (gmem(on_device=True)), else None."""
        return self.__dict__.get("_gmem")

    def gmem(self, on_device=False):
        """Memory kernel K_i = gamt(dt*i) for i < ml (baths.py:412-445).

        on_device (extension): keep only the coefficient matrix W of gmem_coefficients and the
        spectrum; the kernel itself is built in HBM by gle_add_bath_gmem (no host copy of the
        ml x nc x nc kernel, no PCIe transfer)."""
        if self.ml is None or self.dt is None:
            raise ValueError("phbath.gmem: length of memory kernel not set")
        if self.local:
            self.ml = 1
            self.kernel = self.gamma
            return
        tl = [self.dt * i for i in range(self.ml)]
        if on_device:
            gam = np.asarray(self.gamma, dtype=float)
            W = gmem_coefficients(tl, self.wl, self.gwl, self.eta_ad)
            self.kernel = None
            self.__dict__["_gmem"] = (W, gam)
            if self.eta_ad != 0:
                # gamma update of baths.py:429-445: sum_it dt K[it] cos(gwl t_it) = (D . W) . gamma
                d = np.cos(np.outer(np.asarray(self.gwl, dtype=float), np.asarray(tl))) * self.dt
                g = (d @ W) @ gam.reshape(len(gam), -1)
                self.gammaOld = self.gamma
                self.gamma = np.real(g).reshape(np.shape(self.gammaOld))
            return
        self.kernel = gamt(tl, self.wl, self.gwl, self.gamma, self.eta_ad)
        if self.eta_ad != 0:
            c = np.cos(np.outer(np.asarray(self.gwl, dtype=float), np.asarray(tl))) * self.dt
            g = c @ self.kernel.reshape(len(tl), -1)
            self.gammaOld = self.gamma
            self.gamma = np.real(g).reshape(np.shape(self.gammaOld))

    def _noise_key(self):
        return ("ph", self.T, self.wmax, self.dt, self.nmd, self.classical, self.zpmotion,
                _digest(self.gamma, self.gwl))

    def _spectrum(self):
        return _noise.phonon_spectrum(self.gamma, self.gwl, self.T, self.wmax, self.dt, self.nmd,
                                      self.classical, self.zpmotion)

    # streamed factors (noise.stream_factor_chunks): A(w) = Delta equ(w) flinterp(w, gwl, gamma),
    # hermitianised (noise.py:73-79); where flinterp returns a node (its flat end half-cells,
    # functions.py:124-127) A is a non-negative multiple of that node's matrix
    def _shared_matrices(self):
        from .functions import hermitianize

        g = np.asarray(self.gamma)
        return [(0, hermitianize(g[0])), (len(g) - 1, hermitianize(g[-1]))]

    def _spectrum_term(self, i, matrix=True):
        """(kind, shared key, scale, dense matrix or None) of frequency i; matrix=False classifies
        without building the dense matrix."""
        from .functions import flinterp, hermitianize, nearest

        dw = 2.0 * np.pi / self.dt / self.nmd
        delta = self.dt * self.nmd
        w = dw * i
        c = delta * _noise.equ(w, self.wmax, self.T, self.classical, self.zpmotion)
        if c == 0.0:
            return "zero", None, 0.0, None
        n = nearest(w, self.gwl)
        if n == 0 or n == len(self.gwl) - 1:
            return "shared", (0 if n == 0 else len(self.gwl) - 1), float(c), None
        return "dense", None, 1.0, hermitianize(c * flinterp(w, self.gwl, self.gamma)) if matrix else None
