"""The shape of the reference's examples/current-induced/rundp.py through the drop-in API: 242 atoms,
nmd = 2 10^5 (not a power of two), three electron baths (two unbiased friction baths of 120 DOFs,
one biased bath of 36 DOFs with exim / exip), fixed atoms, noranvel, power spectra with a power
section, SaveTraj.  The potential is a harmonic chain on the device (the example's DeePMD / LAMMPS
driver is absent here: parity of the host-driver path is tested elsewhere), the biased bath's
eta / xim / xip matrices are synthetic (the example reads them from grapheneLambda-r-0.3-ver2.nc).
Prints one JSON line: the phases' wall times and the run's kappa.

    python scripts/rundp_shape.py [--nmd N] [--out file.json]"""
import argparse
import json
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nmd", type=int, default=2 * 10 ** 5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    out = os.path.abspath(a.out) if a.out else None
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic
    from sclmd_amd.baths import ebath

    natom = 242
    T, delta, dt, nmd = 300.0, 0.0, 0.5 / 0.658, a.nmd
    dyn = synthetic.chain_dyn(natom)
    fixatoms = [range(0 * 3, (7 + 1) * 3), range(226 * 3, (241 + 1) * 3)]
    slist = list(range(111 * 3, (122 + 1) * 3))
    ecatsl = list(range(8 * 3, (47 + 1) * 3))
    ecatsr = list(range(186 * 3, (225 + 1) * 3))
    rng = np.random.default_rng(3)
    damp = 100 / 0.658211814201041
    n = len(slist)
    s = 1e-3 / damp
    eta = np.eye(n) / damp + s * synthetic.spd(n, rng)
    xim = rng.normal(size=(n, n)) * s
    xip = rng.normal(size=(n, n)) * s
    os.chdir(tempfile.mkdtemp())
    t0 = time.perf_counter()
    mdrun = MD.md(dt, nmd, T, syslist=None, axyz=synthetic.axyz_chain(natom), dyn=dyn, nstart=0, nstop=1,
                  noise_mode="device", verbose=False)
    mdrun.AddBath(ebath(ecatsl, T * (1 - delta / 2), mdrun.dt, mdrun.nmd, wmax=2., nw=1000, bias=0,
                        efric=(1.0 / damp) * np.identity(len(ecatsl)), classical=False, zpmotion=False))
    mdrun.AddBath(ebath(ecatsr, T * (1 - delta / 2), mdrun.dt, mdrun.nmd, wmax=2., nw=1000, bias=0,
                        efric=(1.0 / damp) * np.identity(len(ecatsr)), classical=False, zpmotion=False))
    mdrun.AddBath(ebath(slist, T * (1 + delta / 2), mdrun.dt, mdrun.nmd, wmax=2., nw=1000, bias=1.0, efric=eta,
                        exim=xim, exip=xip, zeta1=None, zeta2=None, classical=False, zpmotion=False))
    mdrun.AddConstr(fixatoms)
    mdrun.noranvel()
    mdrun.CalPowerSpec()
    mdrun.AddPowerSection([ecatsl, slist, ecatsr])
    mdrun.SaveTraj(1000)
    mdrun.Run()
    wall = time.perf_counter() - t0
    kap = np.array(mdrun.kappa_runs).tolist()
    phases = dict(getattr(mdrun, "phase_times", {}) or {})
    ok = bool(np.all(np.isfinite(np.asarray(mdrun.q))) and np.all(np.isfinite(np.asarray(mdrun.power))))
    mdrun.close()
    line = {"nmd": nmd, "natom": natom, "baths": [len(ecatsl), len(ecatsr), len(slist)], "wall_s": round(wall, 2),
            "steps_per_s_wall": round(nmd / wall, 1), "phases_s": phases,
            "kappa_runs": kap, "finite": ok}
    print(json.dumps(line), flush=True)
    if out:
        with open(out, "w") as f:
            f.write(json.dumps(line) + "\n")


if __name__ == "__main__":
    main()
