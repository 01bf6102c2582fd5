#!/usr/bin/env python3
"""C1 host-driver step timing: examples/runmd.py's system (201 atoms, 2 electron
baths nc=150, fixed ends) with the host force driver called every step, one run of NMD steps.
Splits the wall time into driver calls (host) and the rest (device step + transfers).  Prints one
JSON line.  Run on the GPU box:  python scripts/c1_driver_timing.py --nmd 1024"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nmd", type=int, default=1024)
    args = ap.parse_args()
    from sclmd_amd.baths import ebath
    from sclmd_amd.drivers import HarmonicDriver
    from sclmd_amd.md import md
    from sclmd_amd.synthetic import axyz_chain, chain_dyn

    T, delta, dt, nmd = 300, 0.1, 0.25 / 0.658, args.nmd
    lmp = HarmonicDriver(chain_dyn(201), axyz_chain(201))
    t_drv = [0.0]
    force = lmp.force

    def timed_force(q):
        t0 = time.perf_counter()
        f = force(q)
        t_drv[0] += time.perf_counter() - t0
        return f

    lmp.force = timed_force
    fixatoms = [range(0, 60), range(181 * 3, 201 * 3)]
    ecatsl, ecatsr = range(60, 210), range(393, 543)
    m = md(dt, nmd, T, axyz=lmp.axyz, nstart=0, nstop=1, verbose=False)
    m.AddPotential(lmp)
    damp = 100 / 0.658211814201041
    for cids, Tb in ((ecatsl, T * (1 + delta / 2)), (ecatsr, T * (1 - delta / 2))):
        m.AddBath(ebath(cids, Tb, m.dt, m.nmd, wmax=1., nw=500, bias=0.0,
                        efric=(1.0 / damp) * np.identity(len(cids)), classical=False, zpmotion=True))
    m.AddConstr(fixatoms)
    np.random.seed(1)
    m.initialise()
    m.ResetHis()
    for i in range(len(m.baths)):
        m.gen_noise(i, 0)
    m.steps(16)  # warm-up (device setup, first launches)
    calls0, t_drv[0] = lmp.ncalls, 0.0
    t0 = time.perf_counter()
    m.steps(nmd)
    _ = m.p
    wall = time.perf_counter() - t0
    calls = lmp.ncalls - calls0
    print(json.dumps({"config": "C1: examples/runmd.py shape, 201 atoms (603 DOF), 2 ebaths nc=150, ml=1, "
                                "host harmonic driver (lammpsdriver surface), 1 trajectory",
                      "steps": nmd, "ms_per_step": wall / nmd * 1e3, "steps_per_s": nmd / wall,
                      "driver_calls_per_step": calls / nmd, "driver_ms_per_step": t_drv[0] / nmd * 1e3,
                      "other_ms_per_step": (wall - t_drv[0]) / nmd * 1e3}))
    m.close()


if __name__ == "__main__":
    main()
