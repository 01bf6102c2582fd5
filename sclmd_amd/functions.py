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
