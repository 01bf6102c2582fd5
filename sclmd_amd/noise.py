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
        aw = delta * equ(w, ecut, T, classical, zpmotion)
        awm = delta * equ(U.hbar * w - bias, ecut, T, classical, zpmotion)
        awp = delta * equ(U.hbar * w + bias, ecut, T, classical, zpmotion)
        m = aw * efric
        m = m + (-0.5 * aw * exip + 0.5 * awm * (exip + 1j * exim))
        m = m + (-0.5 * aw * exip + 0.5 * awp * (exip - 1j * exim))
        out[n] = hermitianize(m)
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


def stream_factor_plan(bath, chunk=64, workers=None, cache=None):
    """The streamed factors of a bath as device work segments, in frequency order:
      ("shared", w0, nw, scale, F)  frequencies [w0, w0 + nw) whose spectrum is s_w H for one shared
                                    H: factor F = H_+^(1/2) handed over once, scale = sqrt(s_w)
      ("dense", w0, M)              M (nw, nc, nc) the factors of frequencies [w0, w0 + nw); complex
                                    factors as a pair (Re M, Im M) of contiguous planes
    Frequencies whose spectrum is zero produce nothing (the device spectrum starts at zero).  Dense
    factors are computed on a thread pool (LAPACK releases the GIL; BLAS pinned to one thread per
    worker), two chunks ahead of the consumer.  cache: a dict that keeps the dense chunks (and the
    shared factors) of this bath across runs -- the factors do not change between runs, only the
    draws (md.py:569-570) -- so later runs hand over the cached factors without factorising."""
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
