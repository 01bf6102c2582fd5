"""Synthetic junctions of the shapes BASELINE.json names.

There is no network for real LAMMPS/REBO inputs, so the benchmark and the large parity tests use
seeded synthetic systems: a 1-D harmonic chain (nearest-neighbour spring k on every Cartesian axis
plus an on-site term) and per-bath friction spectra Gamma(w) = g0 * A * exp(-(w/wc)^2) with a
random SPD A, turned into memory kernels with phbath.gmem exactly as a user would.
"""
import numpy as np

from .baths import ebath, phbath

DT = 0.25 / 0.658        # examples/runmd.py:23
G0 = 0.658 / 100.0       # 1 / (100 fs) friction scale (runmd.py:46)


def chain_dyn(natom, k=0.01, onsite=1e-3):
    n = 3 * natom
    d = np.zeros((n, n))
    idx = np.arange(n)
    d[idx, idx] = onsite
    for a in range(natom - 1):
        for x in range(3):
            i, j = 3 * a + x, 3 * (a + 1) + x
            d[i, i] += k
            d[j, j] += k
            d[i, j] -= k
            d[j, i] -= k
    return d


def axyz_chain(natom, el="C", spacing=1.42):
    return [[el, spacing * a, 0.0, 0.0] for a in range(natom)]


def spd(n, rng, scale=1.0):
    r = rng.normal(size=(n, n))
    return scale * (r @ r.T / n + np.eye(n))


def gamma_spectrum(nc, rng, ngw=101, wmax=0.5, wc=0.1):
    gwl = np.linspace(0.0, wmax, ngw)
    A = spd(nc, rng)
    env = G0 * np.exp(-(gwl / wc) ** 2)
    return gwl, env[:, None, None] * A[None]


CONFIGS = {
    # name: (natom, phonon-bath atom ranges, ml, nmd, ebath atom range or None)
    "C2": (300, [(0, 100), (200, 300)], 1024, 4096, None),
    "C3": (300, [(0, 100), (200, 300)], 1024, 4096, None),
    "C5": (1000, [(0, 333), (667, 1000)], 4096, 8192, (333, 667)),
}


def make_phbath(T, dofs, ml, nmd, rng, dt=DT, nw=500, debye=0.2, gmem_device=False):
    gwl, gam = gamma_spectrum(len(dofs), rng)
    b = phbath(T, dofs, debye=debye, nw=nw, dt=dt, nmd=nmd, ml=ml, mcof=2.0, gamma=gam, gwl=gwl)
    b.gmem(on_device=gmem_device)
    return b


def make_biased_ebath(T, dofs, nmd, rng, dt=DT, bias=1.0):
    n = len(dofs)
    s = 1e-3 * G0

    def anti():
        r = rng.normal(size=(n, n)) * s
        return r - r.T

    def sym():
        r = rng.normal(size=(n, n)) * s
        return r + r.T

    return ebath(dofs, T, dt, nmd, wmax=1.0, nw=500, bias=bias, efric=G0 * (np.eye(n) + 0.1 * spd(n, rng)),
                 exim=anti(), exip=sym(), zeta1=sym(), zeta2=anti())


def junction(config="C3", T=300.0, delta=0.1, seed=1234, ml=None, nmd=None, natom=None, nw=500,
             gmem_device=False):
    """(dyn, axyz, baths, meta) for a configuration; ml/nmd/natom override the defaults for
    reduced test sizes.  Bath temperatures T(1 +- delta/2) as in runmd.py:51-55.  gmem_device:
    phonon-bath kernels are built on the device (phbath.gmem(on_device=True))."""
    na, ranges, ml0, nmd0, erange = CONFIGS[config]
    natom = natom or na
    scale = natom / na
    ml = ml or ml0
    nmd = nmd or nmd0
    rng = np.random.default_rng(seed)
    dyn = chain_dyn(natom)
    baths = []
    temps = [T * (1 + delta / 2), T * (1 - delta / 2)]
    for (a0, a1), Tb in zip(ranges, temps):
        a0, a1 = int(round(a0 * scale)), int(round(a1 * scale))
        dofs = list(range(3 * a0, 3 * a1))
        baths.append(make_phbath(Tb, dofs, ml, nmd, rng, nw=nw, gmem_device=gmem_device))
    if erange is not None:
        a0, a1 = int(round(erange[0] * scale)), int(round(erange[1] * scale))
        baths.append(make_biased_ebath(T, list(range(3 * a0, 3 * a1)), nmd, rng))
    meta = {"config": config, "natom": natom, "nph": 3 * natom, "ml": ml, "nmd": nmd, "T": T,
            "delta": delta, "dt": DT, "nc": [b.nc for b in baths]}
    return dyn, axyz_chain(natom), baths, meta
