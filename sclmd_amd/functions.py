"""Host numerical helpers with sclmd's conventions (sclmd/functions.py).  Setup-time only: the
per-step arithmetic runs on the device."""
import numpy as np

from . import units as U


def bose(w, T):
    """Bose occupation; bose(0, T>0) = 0 and the T = 0 branches of functions.py:80-99."""
    if T == 0.0:
        if w == 0.0:
            with np.errstate(over="ignore"):
                return 1.0 / (np.exp(1.0 / U.kb) - 1.0)
        return -1.0 if w < 0.0 else 0.0
    if w == 0.0:
        return 0.0
    with np.errstate(over="ignore"):
        return 1.0 / (np.exp(w / U.kb / T) - 1.0)


def coth(x):
    """Hyperbolic cotangent (functions.py:59-67); coth(0) raises (the reference exits)."""
    if x == 0.0:
        raise ValueError("coth: coth(0) is infinite")
    return np.cosh(x) / np.sinh(x)


def xcoth(x):
    """x coth(x), 1 at x = 0 (functions.py:70-77)."""
    return 1.0 if x == 0.0 else x * np.cosh(x) / np.sinh(x)


def fermi(ep, mu, T):
    """Fermi occupation; at T = 0 a step with 1/2 at ep = mu (functions.py:102-114)."""
    if T == 0.0:
        return 1.0 if ep < mu else (0.0 if ep > mu else 0.5)
    with np.errstate(over="ignore"):
        return 1.0 / (np.exp((ep - mu) / U.kb / T) + 1.0)


def nearest(b, bs):
    """Index of the first element of bs closest to b (functions.py:137-143)."""
    return int(np.argmin(np.abs(np.asarray(bs) - b)))


def interp_weights(x, xs):
    """(i, j, wi, wj) such that flinterp(x, xs, ys) == wi*ys[i] + wj*ys[j] (functions.py:117-134):
    linear interpolation from the NEAREST node towards the neighbour on x's side; flat at the
    first and last node."""
    i = nearest(x, xs)
    n = len(xs)
    if i == n - 1 or i == 0:
        return i, i, 1.0, 0.0
    dd = x - xs[i]
    j = i - 1 if dd < 0 else i + 1
    c = dd / (xs[i] - xs[j])
    return i, j, 1.0 + c, -c


def flinterp(x, xs, ys):
    i = nearest(x, xs)
    if i == len(xs) - 1:
        return ys[-1]
    if i == 0:
        return ys[0]
    dd = x - xs[i]
    j = i - 1 if dd < 0 else i + 1
    return ys[i] + dd / (xs[i] - xs[j]) * (ys[i] - ys[j])


def flinterp_many(xq, xs, ys):
    """flinterp at every point of xq, returned as an array (len(xq), *ys.shape[1:])."""
    ys = np.asarray(ys)
    return np.array([flinterp(x, xs, ys) for x in xq])


def chkShape(a):
    a = np.asarray(a)
    if a.ndim != 2 or a.shape[0] != a.shape[1]:
        raise ValueError("the matrix should be an n by n matrix, got shape %s" % (a.shape,))
    return a.shape[0]


def symmetrize(a):
    a = np.asarray(a)
    return 0.5 * (a + a.T)


def antisymmetrize(a):
    a = np.asarray(a)
    return 0.5 * (a - a.T)


def dagger(a):
    """Conjugate transpose of a square matrix (functions.py:189-195)."""
    a = np.asarray(a)
    if a.ndim != 2 or a.shape[0] != a.shape[1]:
        raise ValueError("dagger: not a square matrix")
    return np.conjugate(a).T


def mm(*args):
    """Left-to-right product of any number of matrices (functions.py:159-163)."""
    out = np.array(args[0], copy=True)
    for m in args[1:]:
        out = np.dot(out, m)
    return out


def hermitianize(a):
    a = np.asarray(a)
    return 0.5 * (a + np.conj(np.swapaxes(a, -1, -2)))


def mdot(*args):
    return np.linalg.multi_dot(list(args)) if len(args) > 2 else np.dot(args[0], args[1])


def rpadleft(bs, b):
    """Push b in front of the history bs and drop the oldest row (functions.py:146-153)."""
    bs = np.asarray(bs)
    if len(bs) < 1:
        raise ValueError("empty history")
    return np.concatenate((np.asarray(b)[None], bs[:-1]), axis=0)


class myfft:
    """sclmd's Fourier conventions (functions.py:11-53): t->w is ifft*2pi/dw, w->t is fft*dw/2pi."""

    def __init__(self, dt, n):
        self.dt, self.N = dt, n
        self.dw = 2 * np.pi / dt / n

    def Fourier1D(self, a):
        if len(a) != self.N:
            raise ValueError("myfft.Fourier1D: array length error")
        return (2.0 * np.pi / self.dw) * np.fft.ifft(a)

    def iFourier1D(self, a):
        if len(a) != self.N:
            raise ValueError("myfft.iFourier1D: array length error")
        return (self.dw / 2 / np.pi) * np.fft.fft(a)


def powerspecp(ps, dt, nmd):
    """Velocity power spectrum summed over DOFs (functions.py:221-236): rows [w_i, P(w_i)]."""
    ps = np.asarray(ps)
    if ps.shape[0] != nmd:
        raise ValueError("power: ps shape error")
    dw = 2.0 * np.pi / dt / nmd
    spec = (2.0 * np.pi / dw) * np.fft.ifft(ps, axis=0)
    pw = np.real(spec * np.conj(spec)).sum(axis=1) / dt / nmd
    return np.column_stack((dw * np.arange(nmd), pw))


def powerspecq(qs, dt, nmd):
    """Displacement power spectrum summed over DOFs (functions.py:203-218): rows [w_i, w_i^2 P_q(w_i)]
    with P_q = sum_k |Fourier1D(qs[:, k])|^2 / (dt nmd)."""
    qs = np.asarray(qs)
    if qs.shape[0] != nmd:
        raise ValueError("power: qs shape error")
    dw = 2.0 * np.pi / dt / nmd
    spec = (2.0 * np.pi / dw) * np.fft.ifft(qs, axis=0)
    w = dw * np.arange(nmd)
    return np.column_stack((w, w ** 2 * np.real(spec * np.conj(spec)).sum(axis=1) / dt / nmd))
