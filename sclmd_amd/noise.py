"""Quantum coloured noise (sclmd/noise.py) -- host spectral factorisation + device generation.

The reference draws, for each of the nmd/2+1 positive frequencies w_i, a Gaussian vector with
covariance A(w_i) (eigh + vargau, noise.py:73-84 / 171-191), mirrors the amplitudes into a
length-nmd spectrum (noise.py:87-94) and transforms w -> t with numpy's forward FFT times dw/2pi
(functions.py:36-53).  Here:

  * the covariance matrices A(w_i) and their eigendecompositions are built on the host once per
    bath (they do not change between runs; numpy's eigh on the stacked matrices is the same
    LAPACK call the reference makes one frequency at a time);
  * the Gaussian draws are either numpy-compatible (same legacy RandomState calls in the same
    order as vargau, so seeded runs reproduce the reference draw for draw) or counter-based Philox
    on the device (ensemble mode);
  * the matrix products a_w = U_w r_w, the mirroring and the FFT run in HIP (gle_noise_generate).
"""
import numpy as np

from . import _native
from . import units as U
from .functions import flinterp, hermitianize


def mf(f, cats, lens):
    """Scatter a bath-local vector into the full DOF space (noise.py:15-22)."""
    t = np.zeros(lens)
    t[np.asarray(cats, dtype=int)] = f
    return t


def equ(w, cut, T, classical=False, zpmotion=True):
    """2*hw*(zp + bose(hw,T)) below the cutoff, 2kT classically or at w = 0 (noise.py:249-270)."""
    from .functions import bose

    hw = U.hbar * w
    zp = 0.5 if zpmotion is True else 0.0
    if hw < cut:
        if classical or hw == 0:
            return 2.0 * U.kb * T
        return 2.0 * hw * (zp + bose(hw, T))
    return 0.0


def _neq(w, bias, T, classical, sign):
    """2 (hw + sign bias) (bose(hw + sign bias) - bose(hw)); classically kT / x with x = 0 moved to
    1e-19 (noise.py:211-246)."""
    from .functions import bose

    h1, h2 = U.hbar * w + sign * bias, U.hbar * w
    if classical:
        h1 = h1 if h1 != 0.0 else 10e-20
        h2 = h2 if h2 != 0.0 else 10e-20
        return 2.0 * h1 * (U.kb * T / h1 - U.kb * T / h2)
    return 2.0 * h1 * (bose(h1, T) - bose(h2, T))


def nonequm(w, bias, T, classical=False):
    """Non-equilibrium electron occupation factor at hw - bias (noise.py:211-227)."""
    return _neq(w, bias, T, classical, -1.0)


def nonequp(w, bias, T, classical=False):
    """Non-equilibrium electron occupation factor at hw + bias (noise.py:230-246)."""
    return _neq(w, bias, T, classical, 1.0)


def phnoisew(gamma, wl, T, phcut, classical=False, zpmotion=True):
    """Phonon noise spectrum on the frequencies wl: equ(w_i) gamma[i] (noise.py:28-47)."""
    gamma = np.asarray(gamma)
    out = np.zeros(gamma.shape, dtype=np.result_type(gamma, np.float64))
    for i, w in enumerate(wl):
        out[i] = equ(w, phcut, T, classical, zpmotion) * gamma[i]
    return out


def _electron_matrix(w, efric, exim, exip, bias, T, ecut, scale, classical, zpmotion):
    """Hermitian part of the electron-bath spectral matrix at w, times `scale` (noise.py:172-186)."""
    aw = scale * equ(w, ecut, T, classical, zpmotion)
    awm = scale * equ(U.hbar * w - bias, ecut, T, classical, zpmotion)
    awp = scale * equ(U.hbar * w + bias, ecut, T, classical, zpmotion)
    m = aw * efric
    m = m + (-0.5 * aw * exip + 0.5 * awm * (exip + 1j * exim))
    m = m + (-0.5 * aw * exip + 0.5 * awp * (exip - 1j * exim))
    return hermitianize(m)


def enoisew(wl, efric, exim, exip, bias, T, ecut, classical=False, zpmotion=True):
    """Electron noise spectrum on the frequencies wl (noise.py:105-146: the same matrix as enoise's
    without the Delta = dt nmd factor).  (The reference's own enoisew raises before computing: its
    local `np = chkShape(exip)` shadows numpy, noise.py:122-128.)"""
    efric, exim, exip = (np.asarray(m, dtype=float) for m in (efric, exim, exip))
    if not (efric.shape == exim.shape == exip.shape and efric.shape[0] == efric.shape[1]):
        raise ValueError("enoisew: efric / exim / exip shape error")
    out = np.empty((len(wl),) + efric.shape, dtype=complex)
    for n, w in enumerate(wl):
        out[n] = _electron_matrix(w, efric, exim, exip, bias, T, ecut, 1.0, classical, zpmotion)
    return out


def vargau(eval, evec, cof=1.0):
    """One multivariate Gaussian draw U r, r_k ~ N(0, sqrt(cof lambda_k)) for cof lambda_k > 0 (0
    otherwise), from the global numpy RNG in eigenvalue order (noise.py:273-305).  The generators
    draw all frequencies at once with the same sequence (NoiseFactor.draws)."""
    evec = np.asarray(evec)
    if evec.ndim != 2 or evec.shape[0] != evec.shape[1] or len(eval) != evec.shape[0]:
        raise ValueError("vargau: shape error")
    r = [np.random.normal(0.0, np.sqrt(cof * v)) if cof * v > 0 else 0.0 for v in eval]
    return np.linalg.multi_dot([evec, r]) if len(r) > 1 else evec @ np.asarray(r)


def frequencies(dt, nmd):
    hlen = int(nmd / 2)
    dw = 2.0 * np.pi / dt / nmd
    return dw * np.arange(hlen + 1), dt * nmd


def phonon_spectrum(gamma, wl, T, phcut, dt, nmd, classical=False, zpmotion=True):
    """A(w_i) = Delta*equ(w_i)*Gamma(w_i), hermitianised (noise.py:73-79).  (nfreq, nc, nc)."""
    ws, delta = frequencies(dt, nmd)
    gamma = np.asarray(gamma)
    out = np.empty((len(ws),) + gamma.shape[1:], dtype=np.result_type(gamma, np.float64))
    for n, w in enumerate(ws):
        out[n] = hermitianize(delta * equ(w, phcut, T, classical, zpmotion) * flinterp(w, wl, gamma))
    return out


def electron_spectrum(efric, exim, exip, bias, T, ecut, dt, nmd, classical=False, zpmotion=True):
    """Complex Hermitian A(w_i) of the (biased) electron bath (noise.py:171-186)."""
    ws, delta = frequencies(dt, nmd)
    efric, exim, exip = (np.asarray(m, dtype=float) for m in (efric, exim, exip))
    out = np.empty((len(ws),) + efric.shape, dtype=complex)
    for n, w in enumerate(ws):
        out[n] = _electron_matrix(w, efric, exim, exip, bias, T, ecut, delta, classical, zpmotion)
    return out


class NoiseFactor:
    """Eigendecomposition of a bath's noise spectrum, shared by every run and trajectory."""

    def __init__(self, spectrum):
        spectrum = np.asarray(spectrum)
        self.nfreq, self.nc = spectrum.shape[0], spectrum.shape[1]
        ev, vec = np.linalg.eigh(spectrum)
        self.evals = ev                     # (nfreq, nc) ascending
        self.evecs = vec                    # (nfreq, nc, nc) columns
        self.pos = ev > 0                   # vargau draws only for positive eigenvalues
        self.sigma = np.sqrt(np.where(self.pos, ev, 0.0))
        self.complex = np.iscomplexobj(vec)

    def scaled(self):
        """U.diag(sqrt(max(lambda, 0))) -- the factor for device N(0,1) draws."""
        return self.evecs * self.sigma[:, None, :]

    def draws(self, rng=None):
        """vargau's r vectors for every frequency (noise.py:297-303): N(0, sqrt(lambda_k)) for
        lambda_k > 0 in (frequency, ascending-eigenvalue) order, 0 otherwise.  One vectorised call
        of the legacy RandomState.normal yields the same sequence as the reference's scalar calls."""
        rng = np.random if rng is None else rng
        r = np.zeros((self.nfreq, self.nc))
        s = self.sigma[self.pos]
        if s.size:
            r[self.pos] = rng.normal(0.0, s)
        return r


# ---------------------------------------------------------------------------------------------
# streamed factors (baths whose nfreq x nc x nc factors do not fit on the device, e.g. C5)
def positive_factor(a):
    """U diag(sqrt(max(lambda, 0))) of a Hermitian matrix: the covariance vargau draws from
    (noise.py:273-305, only positive eigenvalues)."""
    ev, vec = np.linalg.eigh(a)
    return vec * np.sqrt(np.where(ev > 0, ev, 0.0))[None, :]


def dense_factor(a):
    """A factor M with M M^H = A_+ for one frequency.  Real symmetric positive-definite A: its
    Cholesky factor (the same Gaussian distribution as the eigen factor for real draws, at ~1/10 of
    the cost); otherwise (complex Hermitian, or not positive definite) the eigen factor, so complex
    baths keep the reference's eigenvector phases."""
    if not np.iscomplexobj(a):
        try:
            return np.linalg.cholesky(a)
        except np.linalg.LinAlgError:
            pass
    return positive_factor(a)


def stream_factor_chunks(bath, chunk=64, workers=None):
    """Yield (w0, M) with M (nw, nc, nc) the factors of frequencies [w0, w0 + nw), built on a
    thread pool (LAPACK releases the GIL; BLAS pinned to one thread per worker).  The bath supplies
    per frequency either nothing (A = 0), a shared matrix with a non-negative scale (A = s H: factor
    sqrt(s) H_+^(1/2), one eigendecomposition for all such frequencies) or the dense A."""
    import os
    from concurrent.futures import ThreadPoolExecutor

    from threadpoolctl import threadpool_limits

    nfreq = int(bath.nmd / 2) + 1
    nc = bath.nc
    cplx = bath.kind == "ebath"
    dtype = complex if cplx else float
    shared = {}
    if workers is None:
        try:
            workers = len(os.sched_getaffinity(0))
        except AttributeError:  # pragma: no cover
            workers = os.cpu_count() or 1
        workers = max(1, min(16, workers))

    def one(i):
        kind, key, s, a = bath._spectrum_term(i)
        if kind == "zero":
            return np.zeros((nc, nc), dtype=dtype)
        if kind == "shared":
            return np.sqrt(s) * shared[key]
        return dense_factor(a).astype(dtype, copy=False)

    with threadpool_limits(1, user_api="blas"), ThreadPoolExecutor(max_workers=workers) as pool:
        for key, h in bath._shared_matrices():
            shared[key] = positive_factor(h).astype(dtype, copy=False)
        futs = []
        for w0 in range(0, nfreq, chunk):
            futs.append((w0, [pool.submit(one, i) for i in range(w0, min(nfreq, w0 + chunk))]))
            if len(futs) > 2:  # two chunks in flight ahead of the device
                w, fl = futs.pop(0)
                yield w, np.stack([f.result() for f in fl])
        for w, fl in futs:
            yield w, np.stack([f.result() for f in fl])


class NodeShare:
    """The ranks of one node factorising a bath's noise spectrum together (the factors
    are the same on every rank, only the draws differ): rank r computes the dense factors of its
    contiguous block of the dense frequencies and publishes them as two node-local shared-memory
    files (the factors, [planes][n][nc][nc] float64, then their frequency indices); after a barrier
    every rank maps every block and hands the factors to its device in frequency order.  Each
    factor is computed once on the node, by the same single-threaded LAPACK call one rank would
    make, so every rank's factors -- and noise -- are bitwise those of one rank factorising alone.
    A block whose files are missing after the barrier (a rank on another node) is computed locally.

    barrier(): a collective over the ranks (md: a one-double all-reduce of its process group or
    C-ABI communicator); token: the same string on every rank and unique to the job (md: rank 0's
    random number, summed over the ranks)."""

    def __init__(self, rank, world, barrier, token, root=None):
        import os

        self.rank, self.world, self.barrier, self.token = int(rank), int(world), barrier, str(token)
        self.root = root or os.environ.get("SCLMD_SHM_DIR", "/dev/shm")
        self.computed = 0   # factorisations this rank computed in the last plan / gather
        self.total = 0      # ... and over every plan / gather so far

    def gather(self, key, n, compute):
        """Arrays over the range [0, n) computed in blocks across the ranks: compute(lo, hi) returns a
        tuple of arrays with hi - lo rows each; every rank gets the tuple concatenated over [0, n)."""
        import os

        lo, hi = self.block(n)
        mine = tuple(compute(lo, hi))
        self.computed = hi - lo
        self.total += hi - lo
        base = os.path.join(self.root, "sclmd_%s_%s_r%%d" % (self.token, key))
        files = ["%s.%d.npy" % (base % self.rank, k) for k in range(len(mine))] + [base % self.rank + ".done"]
        try:
            for f, a in zip(files, mine):
                np.save(f + ".tmp.npy", a)
                os.replace(f + ".tmp.npy", f)
            open(files[-1], "w").close()  # written last: the block is complete
        except OSError:  # no room in shared memory: the other ranks compute this block themselves
            for f in files:
                for g in (f, f + ".tmp.npy"):
                    if os.path.exists(g):
                        os.remove(g)
        self.barrier()
        parts = []
        for r in range(self.world):
            if r == self.rank:
                parts.append(mine)
            elif os.path.exists(base % r + ".done"):
                parts.append(tuple(np.load("%s.%d.npy" % (base % r, k)) for k in range(len(mine))))
            else:
                parts.append(tuple(compute(*self.block(n, r))))
        out = tuple(np.concatenate([p[k] for p in parts]) for k in range(len(mine)))
        self.barrier()  # every rank has read every block
        for f in files:
            if os.path.exists(f):
                os.remove(f)
        return out

    def block(self, n, r=None):
        r = self.rank if r is None else r
        return n * r // self.world, n * (r + 1) // self.world

    def paths(self, key, r):
        import os

        base = os.path.join(self.root, "sclmd_%s_%s_r%d" % (self.token, key, r))
        return base + ".fac.npy", base + ".idx.npy"


def _dense_factors(bath, idx, dtype, workers):
    """Dense factors of frequencies idx on a thread pool (BLAS one thread per worker)."""
    from concurrent.futures import ThreadPoolExecutor

    from threadpoolctl import threadpool_limits

    with threadpool_limits(1, user_api="blas"), ThreadPoolExecutor(max_workers=workers) as pool:
        return list(pool.map(lambda i: dense_factor(bath._spectrum_term(i)[3]).astype(dtype, copy=False), idx))


def _shared_plan(bath, chunk, workers, cache, share, terms, runs, dtype):
    """stream_factor_plan's segments with the dense factors split over the node's ranks (NodeShare)."""
    import os

    nc = bath.nc
    cplx = dtype is complex
    dense = [i for kind, _, ws in runs if kind == "dense" for i in ws]
    import hashlib

    key = "b%s" % hashlib.sha1(repr((bath._noise_key(), chunk)).encode()).hexdigest()[:16]
    a, b = share.block(len(dense))
    mine = dense[a:b]
    fpath, ipath = share.paths(key, share.rank)
    facs = _dense_factors(bath, mine, dtype, workers)
    share.computed = len(mine)
    share.total += len(mine)
    arr = np.empty((2 if cplx else 1, len(mine), nc, nc))
    for k, m in enumerate(facs):
        arr[0, k] = m.real
        if cplx:
            arr[1, k] = m.imag
    del facs
    try:
        np.save(fpath + ".tmp.npy", arr)
        os.replace(fpath + ".tmp.npy", fpath)
        np.save(ipath + ".tmp.npy", np.asarray(mine, dtype=np.int64))
        os.replace(ipath + ".tmp.npy", ipath)  # the index file last: its presence marks the block complete
    except OSError:  # no room in shared memory: the other ranks compute this block themselves
        for f in (fpath, ipath, fpath + ".tmp.npy", ipath + ".tmp.npy"):
            if os.path.exists(f):
                os.remove(f)
    del arr
    share.barrier()
    where = {}  # frequency -> (block array, row)
    blocks = []
    for r in range(share.world):
        fr, ir = share.paths(key, r)
        if os.path.exists(ir):
            idx = np.load(ir)
            fac = np.load(fr, mmap_mode="r")
        else:  # not on this node's shared memory: compute the block here
            lo, hi = share.block(len(dense), r)
            idx = np.asarray(dense[lo:hi], dtype=np.int64)
            fl = _dense_factors(bath, list(idx), dtype, workers)
            fac = np.empty((2 if cplx else 1, len(fl), nc, nc))
            for k, m in enumerate(fl):
                fac[0, k] = m.real
                if cplx:
                    fac[1, k] = m.imag
        blocks.append(fac)
        for k, i in enumerate(idx):
            where[int(i)] = (len(blocks) - 1, k)
    shared = {}
    need = {k for kind, k, _ in runs if kind == "shared"}
    for k, h in bath._shared_matrices():
        if k in need:
            shared[k] = positive_factor(h).astype(dtype, copy=False)
    keep = [] if cache is not None else None
    for kind, k, ws in runs:
        if kind == "shared":
            seg = ("shared", ws[0], len(ws), np.sqrt(np.array([terms[i][2] for i in ws])), shared[k])
        else:
            loc = [where[i] for i in ws]
            bi, r0 = loc[0]
            if all(l == (bi, r0 + j) for j, l in enumerate(loc)):  # one block's contiguous rows: views
                planes = [blocks[bi][p, r0:r0 + len(ws)] for p in range(blocks[bi].shape[0])]
            else:
                planes = [np.stack([blocks[l[0]][p, l[1]] for l in loc]) for p in range(2 if cplx else 1)]
            if keep is not None:  # the host cache outlives the shared files: own copies
                planes = [np.array(x) for x in planes]
            seg = ("dense", ws[0], (planes[0], planes[1]) if cplx else planes[0])
        if keep is not None:
            keep.append(seg)
        yield seg
    share.barrier()  # every rank has handed every block to its device
    for path in share.paths(key, share.rank):
        if os.path.exists(path):
            os.remove(path)
    if cache is not None:
        cache["segments"] = keep
        cache["complete"] = True


def stream_factor_plan(bath, chunk=64, workers=None, cache=None, share=None):
    """The streamed factors of a bath as device work segments, in frequency order:
      ("shared", w0, nw, scale, F)  frequencies [w0, w0 + nw) whose spectrum is s_w H for one shared
                                    H: factor F = H_+^(1/2) handed over once, scale = sqrt(s_w)
      ("dense", w0, M)              M (nw, nc, nc) the factors of frequencies [w0, w0 + nw); complex
                                    factors as a pair (Re M, Im M) of contiguous planes
    Frequencies whose spectrum is zero produce nothing (the device spectrum starts at zero).  Dense
    factors are computed on a thread pool (LAPACK releases the GIL; BLAS pinned to one thread per
    worker), two chunks ahead of the consumer.  cache: a dict that keeps the dense chunks (and the
    shared factors) of this bath across runs -- the factors do not change between runs, only the
    draws (md.py:569-570) -- so later runs hand over the cached factors without factorising.
    share: a NodeShare -- the node's ranks split the dense factorisations and exchange them."""
    import os
    from concurrent.futures import ThreadPoolExecutor

    from threadpoolctl import threadpool_limits

    nfreq = int(bath.nmd / 2) + 1
    nc = bath.nc
    dtype = complex if bath.kind == "ebath" else float
    if cache is not None and cache.get("complete"):
        for seg in cache["segments"]:
            yield seg
        return
    terms = [bath._spectrum_term(i, matrix=False) for i in range(nfreq)]
    # runs: (kind, key, [frequencies])
    runs = []
    for i, (kind, key, sc, _) in enumerate(terms):
        if kind == "zero":
            continue
        if runs and runs[-1][0] == kind and runs[-1][1] == key and runs[-1][2][-1] == i - 1 and \
                (kind == "shared" or len(runs[-1][2]) < chunk):
            runs[-1][2].append(i)
        else:
            runs.append((kind, key, [i]))
    if workers is None:
        try:
            workers = len(os.sched_getaffinity(0))
        except AttributeError:  # pragma: no cover
            workers = os.cpu_count() or 1
        workers = max(1, min(16, workers))
    if share is not None and share.world > 1:
        yield from _shared_plan(bath, chunk, workers, cache, share, terms, runs, dtype)
        return
    keep = [] if cache is not None else None
    shared = {}
    with threadpool_limits(1, user_api="blas"), ThreadPoolExecutor(max_workers=workers) as pool:
        need = {key for kind, key, _ in runs if kind == "shared"}
        for key, h in bath._shared_matrices():
            if key in need:
                shared[key] = positive_factor(h).astype(dtype, copy=False)
        pending = []

        def emit(item):
            kind, key, ws = item
            if kind == "shared":
                sc = np.sqrt(np.array([terms[i][2] for i in ws]))
                seg = ("shared", ws[0], len(ws), sc, shared[key])
            else:
                m = np.stack([f.result() for f in key])
                if np.iscomplexobj(m):  # the device takes real and imaginary planes: split once (and
                    # cache the split), not at every run's hand-over (C5's electron bath: 2 x 4 GB)
                    m = (np.ascontiguousarray(m.real), np.ascontiguousarray(m.imag))
                seg = ("dense", ws[0], m)
            if keep is not None:
                keep.append(seg)
            return seg

        for kind, key, ws in runs:
            if kind == "dense":
                futs = [pool.submit(lambda i=i: dense_factor(bath._spectrum_term(i)[3]).astype(dtype, copy=False))
                        for i in ws]
                pending.append(("dense", futs, ws))
            else:
                pending.append(("shared", key, ws))
            ndense = sum(1 for p in pending if p[0] == "dense")
            while pending and (pending[0][0] == "shared" or ndense > 2):
                if pending[0][0] == "dense":
                    ndense -= 1
                yield emit(pending.pop(0))
        for item in pending:
            yield emit(item)
    if cache is not None:
        cache["segments"] = keep
        cache["complete"] = True


def generate(factor, dt, nmd, ntraj=1, rngs=None, seed=None, device=0):
    """Standalone device generation of ntraj realisations (ntraj, nmd, nc) for one factor."""
    st = _native.Stepper(factor.nc, ntraj, nmd, dt, device)
    try:
        st.add_bath(_native.GLE_BATH_PHONON, np.arange(factor.nc), np.zeros((1, factor.nc, factor.nc)))
        if seed is None:
            st.noise_factors(0, factor.evecs)
            rngs = rngs if rngs is not None else [np.random] * ntraj
            x = np.stack([factor.draws(r) for r in rngs])
            st.noise_generate(0, x)
        else:
            st.noise_factors(0, factor.scaled())
            st.noise_generate(0, None, seed=seed)
        return st.get_noise(0)
    finally:
        st.close()


def phnoise(gamma, wl, T, phcut, dt, nmd, classical=False, zpmotion=True):
    """Phonon-bath noise, same signature and RNG use as noise.py:50-100; returns (nmd, nc) real
    (the reference returns the complex FFT whose real part baths.py:408 keeps)."""
    f = NoiseFactor(phonon_spectrum(gamma, wl, T, phcut, dt, nmd, classical, zpmotion))
    return generate(f, dt, nmd)[0]


def enoise(efric, exim, exip, bias, T, ecut, dt, nmd, classical=False, zpmotion=True):
    """Electron-bath noise, same signature and RNG use as noise.py:149-206; returns (nmd, nc)."""
    f = NoiseFactor(electron_spectrum(efric, exim, exip, bias, T, ecut, dt, nmd, classical, zpmotion))
    return generate(f, dt, nmd)[0]
