#!/usr/bin/env python3
"""Bisect the bench (md path) vs exp_time (Stepper path) step-time gap on one box: the same
device configuration timed after different initial states / noise assignments."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(st, n=512, fill=576):
    st.run(fill)
    st.sync()
    t0 = time.perf_counter()
    st.run(n)
    st.sync()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic

    dyn, axyz, baths, meta = synthetic.junction("C3", seed=1234, gmem_device=True)
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
    p, q, t = st.get_state()
    out = {"thermal_state": timed(st)}
    p2, q2, _ = st.get_state()
    out["p_rms_thermal"] = float(np.sqrt(np.mean(p2 ** 2)))
    out["dq_step_thermal"] = float(np.max(np.abs(p2)) * meta["dt"])
    r = np.random.default_rng(1)
    st.set_state(r.normal(size=(B, meta["nph"])) * 1e-3, r.normal(size=(B, meta["nph"])) * 1e-3, 0)
    for i in range(len(baths)):
        st.set_history(i, None)
    out["random_1e-3_state"] = timed(st)
    st.set_state(p, q, 0)
    for i in range(len(baths)):
        st.set_history(i, None)
    out["thermal_again"] = timed(st)
    out["dt"] = meta["dt"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
