#!/usr/bin/env python3
"""Bisect the bench (md path) vs exp_time (Stepper path) step-time gap: both constructions timed in
one process, in the order Stepper, md, Stepper; then md with exp_time's run sequence."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def timed(st, n=512, fill=576):
    st.run(fill)
    st.sync()
    t0 = time.perf_counter()
    st.run(n)
    st.sync()
    return (time.perf_counter() - t0) / n * 1e6


def expseq(st):
    st.run(517)
    st.sync()
    for n in (20, 3, 20, 64):
        st.run(n)
        st.sync()
    t0 = time.perf_counter()
    st.run(512)
    st.sync()
    return (time.perf_counter() - t0) / 512 * 1e6


def main():
    import exp_time
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic

    dyn, axyz, baths, meta = synthetic.junction("C3", seed=1234, gmem_device=True)

    class A:
        ntraj, steps, short, short_reps, profile = 64, 512, 20, 0, 0

    out = {}
    out["stepper_1"] = exp_time.measure(A, meta, dyn, baths)["ms_per_step"] * 1e3
    B = 64
    m = MD.md(meta["dt"], meta["nmd"], meta["T"], axyz=axyz, dyn=dyn, ntraj=B, seed=1000, traj_offset=0,
              device=0, noise_mode="device", verbose=False)
    for b in baths:
        m.AddBath(b)
    m.initialise()
    m.ResetHis()
    rng = np.random.default_rng(4321)
    for b in baths:
        b.noise = rng.standard_normal((B, meta["nmd"], b.nc)) * 1e-3
    st = m._ensure_device()
    m.steps(0)
    st.sync()
    out["md_1"] = timed(st)
    out["md_expseq"] = expseq(st)
    st.close()
    m._st = None
    out["stepper_2"] = exp_time.measure(A, meta, dyn, baths)["ms_per_step"] * 1e3
    print(json.dumps(out))


if __name__ == "__main__":
    main()
