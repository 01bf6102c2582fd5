"""C1 (BASELINE.json configs[0]): the reference's examples/runmd.py shape run as a script through the
drop-in API -- 201 atoms, two electron baths on DOF 60-209 / 393-542 at T(1 +- delta/2), atoms 0-19 and
181-200 fixed, 3 runs, host force driver called every step -- against the oracle stepping the same
seeded system (ref examples/runmd.py:1-73, md.py:493-665, baths.py:176-192, noise.py:149-206).

LAMMPS/REBO is not in this image: the script's driver is the harmonic stand-in with the
lammpsdriver plugin surface (sclmd_amd/drivers.py), and the oracle calls the same driver.  NMD=256
keeps the oracle to seconds (the script's own default is 2**12).  Tolerances: p/q 1e-9 relative,
per-run time-averaged heat current 1e-9 relative, kappa files to their 6 printed decimals."""
import os
import runpy
import time

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SEED = 2024
NMD = 256


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def _oracle_runmd():
    """md.Run of runmd.py restated with the oracle: no dynamical matrix, so initialise() leaves p = q = 0
    and draws nothing (md.py:298-306); per run, gnoi of bath 0 then bath 1 (md.py:569-570), nmd vv
    steps, kappa = mean(cur) * curcof (md.py:659-664).  History and state carry over between runs."""
    from oracle import sclmd_oracle as O
    from sclmd_amd import units as U
    from sclmd_amd.drivers import HarmonicDriver
    from sclmd_amd.synthetic import axyz_chain, chain_dyn

    T, delta, dt = 300, 0.1, 0.25 / 0.658
    drv = HarmonicDriver(chain_dyn(201), axyz_chain(201))
    fixatoms = [range(0 * 3, (19 + 1) * 3), range(181 * 3, (200 + 1) * 3)]
    ecatsl = np.arange(20 * 3, (69 + 1) * 3)
    ecatsr = np.arange(131 * 3, (180 + 1) * 3)
    damp = 100 / 0.658211814201041
    baths = []
    for cids, Tb in ((ecatsl, T * (1 + delta / 2)), (ecatsr, T * (1 - delta / 2))):
        efric = (1.0 / damp) * np.identity(len(cids))
        baths.append((O.Bath("e", cids, efric[None], None, dt, NMD), efric, Tb))
    sim = O.GLE(603, dt, NMD, [b for b, _, _ in baths], force_fn=drv.force, constr=fixatoms)
    kappa = []
    for _ in range(3):
        for b, efric, Tb in baths:
            z = np.zeros_like(efric)
            b.noise = np.real(O.enoise(efric, z, z, 0.0, Tb, 1.0, dt, NMD, False, True))
        for _ in range(NMD):
            sim.step()
        kappa.append([np.mean(b.cur) * U.curcof for b, _, _ in baths])
    return sim, np.array(kappa)


def test_runmd_script_c1_vs_oracle(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("NMD", str(NMD))
    np.random.seed(SEED)
    t0 = time.perf_counter()
    g = runpy.run_path(os.path.join(ROOT, "examples", "runmd.py"), run_name="__main__")
    wall = time.perf_counter() - t0
    m, drv = g["mdrun"], g["lmp"]
    np.random.seed(SEED)
    sim, kappa = _oracle_runmd()
    assert m.t == sim.t == 3 * NMD
    assert rel(m.p, sim.p) < 1e-9 and rel(m.q, sim.q) < 1e-9
    assert rel(np.array(m.kappa_runs), kappa) < 1e-9
    for j in range(3):
        for i in range(2):
            row = open("kappa.300.bath%d.run%d.dat" % (i, j)).read().split()
            assert int(row[0]) == j and abs(float(row[2]) - kappa[j, i]) < max(2e-6, 1e-9 * abs(kappa[j, i]))
    # the script's own post-processing (tools.calHF / calTC) ran and wrote its tables
    for f in ("heatflux.300.dat", "thermalconductance.300.dat"):
        assert os.path.isfile(f), sorted(os.listdir("."))
    # host-driver path: one (or, on a potential-cache miss, more) driver call per force phase
    steps = 3 * NMD
    assert steps <= drv.ncalls <= 3 * steps + 1
    print("\nC1 runmd.py (201 atoms, 2 ebaths nc=150, host driver): %d steps in %.2f s, %.1f ms/step, "
          "%.2f driver calls/step" % (steps, wall, wall / steps * 1e3, drv.ncalls / steps))
    m.close()
