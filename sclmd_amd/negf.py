"""Ballistic phonon transport by NEGF: the Landauer limit of the GLE ensemble.

Mirrors the public surface of sclmd's `negf.bpt` (negf.py:8-273): transmission `tm`, `gettm`,
`thermalcurrent` / `thermalconductance` / `thermalconductivity`, power spectrum `ps` / `getps`
(optionally with the current-induced bias self-energy, `setbias`), in the reference's units
(frequency in rad/ps, damping time in ps, temperature in K, current in nW).  In the harmonic limit
with time-local (ohmic) baths the semiclassical Langevin ensemble current of `md.Run` must equal
`thermalcurrent`; `tests/test_gpu_negf.py` checks exactly that on the device path.

Differences from the reference, by design:
  * no LAMMPS: the dynamical matrix is passed in (`dynmat=`, the full 3N x 3N matrix in rad^2/ps^2
    as LAMMPS' `dynamical_matrix ... eskm` file holds it, or `dynmatfile=` such a text file);
    `infile` (LAMMPS commands) raises, since the engine is not part of this build;
  * every frequency is evaluated in one batched solve (`numpy.linalg.solve` over a stack of
    matrices) instead of one `inv` per frequency; `vector` is accepted and ignored;
  * no v_sim / matplotlib writers (`write_v_sim`, `plotresult`): visualisation, out of scope.
"""
import numpy as np

RPC = 6.582119569e-4      # hbar, eV ps (negf.py:12)
BC = 8.617333262e-5       # kB, eV/K (negf.py:14)
EV_PER_PS_NW = 1.60217662e2  # eV/ps -> nW (negf.py:267)
_IMAX = float(np.iinfo(np.int32).max)


def _reduced_index(n, fixed):
    """Indices kept after the reference's two-stage deletion of the fixed DOFs (negf.py:198-204):
    fixed[0] is removed first, then fixed[1] shifted down by len(fixed[0])."""
    keep = np.delete(np.arange(n), list(fixed[0]))
    return np.delete(keep, [d - len(fixed[0]) for d in fixed[1]])


class bpt:
    def __init__(self, infile=None, maxomega=0.25, damp=0.1, dofatomofbath=None, dofatomfixed=[[], []],
                 dynmatfile=None, num=1000, *, dynmat=None):
        self.rpc, self.bc = RPC, BC
        self.damp = damp
        self.maxomega = maxomega / self.rpc
        self.intnum = num
        self.dofatomfixed = [list(dofatomfixed[0]), list(dofatomfixed[1])]
        self.isbias = False
        self.dofatomofbias = []
        self.dofatomofbath = [list(dofatomofbath[0]), list(dofatomofbath[1])]
        if dynmat is None and dynmatfile is not None:
            dynmat = np.loadtxt(dynmatfile)
        if dynmat is None:
            raise RuntimeError("bpt: LAMMPS is not part of this build; pass dynmat= or dynmatfile= "
                               "(infile=%r cannot be evaluated)" % (infile,))
        self.getdynmat(dynmat)
        for dofs in self.dofatomofbath:
            self._cols(dofs)  # every bath DOF must be free

    # ------------------------------------------------------------------------------ setup
    def getdynmat(self, dynmat):
        """Symmetrise, drop the fixed DOFs, mode frequencies (negf.py:68-95)."""
        d = np.asarray(dynmat, dtype=float)
        n = int(round(np.sqrt(d.size)))
        if n * n != d.size or n % 3:
            raise ValueError("System DOF test failed after load dynmat, check again")
        d = d.reshape(n, n)
        self.natoms = n // 3
        self.keep = _reduced_index(n, self.dofatomfixed)
        d = (d + d.T) / 2
        self.dynmat = d[np.ix_(self.keep, self.keep)]
        self._pos = {int(g): i for i, g in enumerate(self.keep)}
        ev, self.eigvecs = np.linalg.eigh(self.dynmat)
        self.omegas = np.where(ev > 0, np.sqrt(np.abs(ev)), -np.sqrt(np.abs(ev))) * self.rpc

    def _cols(self, dofs):
        """Reduced positions of full-system DOF indices (every listed DOF must be free)."""
        try:
            return np.array([self._pos[int(d)] for d in dofs], dtype=int)
        except KeyError as e:
            raise ValueError("System DOF test failed, check again (DOF %s is fixed)" % e)

    def setbias(self, bias, bdamp=None, chiplus=None, chiminus=None, dofatomofbias=[]):
        """Current-induced forces on a central region (negf.py:27-39); bias in eV."""
        self.isbias = True
        self.bias = bias / self.rpc
        self.biasgamma = np.asarray(bdamp)
        self.chiplus = np.asarray(chiplus)
        self.chiminus = np.asarray(chiminus)
        self.dofatomofbias = list(dofatomofbias)
        if not (len(self.biasgamma) == len(self.chiminus) == len(self.chiplus) == len(self.dofatomofbias)):
            raise ValueError("Bias parameters not set correctly")

    # ------------------------------------------------------------------------------ self-energies
    def _bath_diag(self, dofs):
        m = np.zeros(len(self.keep))
        m[self._cols(dofs)] = 1.0 / self.damp
        return m

    def _sigma_r(self, w):
        """Retarded self-energy of both baths and the bias region, stacked over w: (nw, n, n)."""
        w = np.atleast_1d(np.asarray(w, dtype=float))
        n = len(self.keep)
        diag = self._bath_diag(self.dofatomofbath[0]) + self._bath_diag(self.dofatomofbath[1])
        s = np.zeros((len(w), n, n), dtype=complex)
        s[:, np.arange(n), np.arange(n)] = -1j * w[:, None] * diag[None, :]
        if self.isbias:
            # block [t1, t2) of the full matrix = the contiguous run first..last bias DOF (negf.py:166-172)
            t1, t2 = self.dofatomofbias[0], self.dofatomofbias[-1] + 1
            c = self._cols(range(t1, t2))
            blk = -1j * w[:, None, None] * self.biasgamma[None] - self.bias * self.chiminus[None]
            s[np.ix_(np.arange(len(w)), c, c)] += blk
        return s

    def _gr(self, w):
        w = np.atleast_1d(np.asarray(w, dtype=float))
        n = len(self.keep)
        a = ((w + 1e-9j) ** 2)[:, None, None] * np.eye(n)[None] - self.dynmat[None] - self._sigma_r(w)
        return np.linalg.solve(a, np.broadcast_to(np.eye(n, dtype=complex), a.shape))

    def retargf(self, omega):
        return self._gr(omega)[0]

    def advangf(self, omega):
        return self.retargf(omega).conj().T

    def gamma(self, Pi):
        return -1j * (Pi - Pi.conj().swapaxes(-1, -2))

    def bosedist(self, omega, T):
        """Bose-Einstein occupation with the reference's T -> 0 and omega/T -> 0 clamps (negf.py:218-228)."""
        if abs(T) < 1e-30:
            with np.errstate(over="ignore", divide="ignore"):
                return 1 / (np.exp(self.rpc * omega * _IMAX) - 1)
        if abs(omega / T) < 1e-30:
            return _IMAX
        return 1 / (np.exp(self.rpc * omega / self.bc / T) - 1)

    def _bose_vec(self, w, T):
        with np.errstate(over="ignore", divide="ignore", invalid="ignore"):
            return np.array([self.bosedist(x, T) for x in np.atleast_1d(w)], dtype=float)

    # ------------------------------------------------------------------------------ transport
    def _tm_vec(self, w):
        """Tr[G^r Gamma_L G^a Gamma_R] over a stack of frequencies (negf.py:237-240)."""
        w = np.atleast_1d(np.asarray(w, dtype=float))
        g = self._gr(w)
        cl = self._cols(self.dofatomofbath[0])
        cr = self._cols(self.dofatomofbath[1])
        # Gamma_b = 2 w / damp on the bath's diagonal: Tr = gamma^2 sum |G^r[R, L]|^2
        gl = 2.0 * w / self.damp
        blk = g[:, cr][:, :, cl]                       # G^r[R, L]
        return (gl * gl) * np.real(np.einsum("wij,wij->w", blk, blk.conj()))

    def tm(self, omega):
        return float(self._tm_vec(omega)[0])

    def gettm(self, vector=False, filename="transmission.dat"):
        x = np.linspace(0, self.maxomega, self.intnum + 1)
        self.tmnumber = np.column_stack((x, self._tm_vec(x)))
        if filename:
            np.savetxt(filename, np.column_stack((self.tmnumber[:, 0] * self.rpc, self.tmnumber[:, 1])))
        return self.tmnumber

    def thermalcurrent(self, T, delta):
        """Landauer current between baths at T(1 +- delta/2), trapezoid over the gettm grid, in nW
        (negf.py:242-267)."""
        if getattr(self, "tmnumber", None) is None:
            self.gettm(filename=None)
        x, t = self.tmnumber[:, 0], self.tmnumber[:, 1]
        n = len(x) - 1
        if n != self.intnum:
            raise ValueError("Error in number of omega")
        with np.errstate(invalid="ignore"):
            f = self.rpc * x / 2 / np.pi * t * (self._bose_vec(x, T * (1 + 0.5 * delta)) -
                                               self._bose_vec(x, T * (1 - 0.5 * delta)))
        return float((x[-1] - x[0]) / n / 2.0 * (2 * f.sum() - f[0] - f[-1])) * EV_PER_PS_NW

    def thermalconductance(self, T, delta):
        return self.thermalcurrent(T, delta) / (T * delta)

    def thermalconductivity(self, T, delta, L, A):
        return self.thermalconductance(T, delta) * L / A * 10

    # ------------------------------------------------------------------------------ power spectrum
    def _sigma_k(self, w, T):
        """Keldysh self-energy of the baths (+ bias region) at one frequency (negf.py:161-194)."""
        n = len(self.keep)
        nb = self.bosedist(w, T)
        diag = self._bath_diag(self.dofatomofbath[0]) + self._bath_diag(self.dofatomofbath[1])
        s = np.diag(2.0 * w * diag * nb).astype(complex)
        if self.isbias:
            t1, t2 = self.dofatomofbias[0], self.dofatomofbias[-1] + 1
            c = self._cols(range(t1, t2))
            wp, wm = w + self.bias, w - self.bias
            semat = ((self.chiplus - 1j * self.chiminus) * wp * (2 * self.bosedist(wp, T) - 2 * nb) +
                     (self.chiplus + 1j * self.chiminus) * wm * (2 * self.bosedist(wm, T) - 2 * nb)) / 2
            sr = -1j * w * self.biasgamma - self.bias * self.chiminus   # Sigma^r of the bias block
            s[np.ix_(c, c)] += 1j * sr * 2 * nb + semat
        return s

    def ps(self, omega, T, atomlist):
        """Power spectrum of the listed DOFs (negf.py:229-235)."""
        c = np.asarray(atomlist) - len(self.dofatomfixed[0])
        g = self.retargf(omega)
        if not self.isbias:
            return float(-2 * omega ** 2 * self.bosedist(omega, T) * np.trace(np.imag(g[np.ix_(c, c)])))
        gk = g @ self._sigma_k(omega, T) @ g.conj().T
        return float(omega ** 2 * np.trace(np.real(gk[np.ix_(c, c)])))

    def getps(self, T, maxomega, intnum, atomlist=None, filename=None, vector=False, omegalist=None):
        if atomlist is None:
            atomlist = np.arange(len(self.dynmat)) + len(self.dofatomfixed[0])
        x2 = (np.sort(omegalist) / self.rpc if omegalist is not None
              else np.linspace(0, maxomega / self.rpc, intnum + 1))
        self.psnumber = np.column_stack((x2, [self.ps(w, T, atomlist) for w in x2]))
        name = ("powerspectrum.%s.%s.dat" % (filename, T)) if filename is not None else "powerspectrum.%s.dat" % T
        np.savetxt(name, np.column_stack((self.psnumber[:, 0] * self.rpc, self.psnumber[:, 1])))
        return self.psnumber

    # ------------------------------------------------------------------------------ md units
    @classmethod
    def from_md(cls, dyn_md, damp_md, dofatomofbath, dofatomfixed=[[], []], maxomega=0.25, num=1000):
        """Junction given in sclmd's md units (units.py: hbar = 1, energies and frequencies in eV,
        time unit 0.658211814201041 fs) with ohmic baths efric = I / damp_md on the bath DOFs."""
        from . import units as U

        time_ps = U.time * 1e12
        return cls(maxomega=maxomega, damp=damp_md * time_ps, dofatomofbath=dofatomofbath,
                   dofatomfixed=dofatomfixed, num=num, dynmat=np.asarray(dyn_md) / RPC ** 2)
