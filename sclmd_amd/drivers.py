"""Host force drivers with the plugin surface of sclmd's lammpsdriver / siestadriver /
deepmddriver (.force(q), .initforce(), .f0, .axyz, .conv, .quit(), .dynmat()).

HarmonicDriver is a stand-in for LAMMPS (not installed here): force(q) = -dyn.q, i.e. the
mass-weighted force relative to the zero-displacement force, exactly what lammpsdriver.force
returns (lammpsdriver.py:83-84) for a harmonic potential."""
import numpy as np

from . import units as U


class HarmonicDriver:
    def __init__(self, dyn, axyz, md2ang=0.06466):
        self.dyn = np.asarray(dyn, dtype=float)
        self.axyz = [list(a) for a in axyz]
        self.md2ang = md2ang
        masses = [U.AtomicMassTable[a[0]] for a in self.axyz]
        self.conv = md2ang * np.array([3 * [1.0 / np.sqrt(m)] for m in masses]).flatten()
        self.xyz = np.array([a[1:] for a in self.axyz], dtype=float).flatten()
        self.ncalls = 0
        self.initforce()

    def absforce(self, q):
        self.ncalls += 1
        return -self.dyn @ np.asarray(q, dtype=float)

    def initforce(self):
        self.f0 = self.absforce(np.zeros(len(self.xyz)))

    def force(self, q):
        return self.absforce(q) - self.f0

    def dynmat(self, q=None):
        return self.dyn.copy()

    def quit(self):
        pass
