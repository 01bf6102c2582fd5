#!/usr/bin/env python3
"""Timing diagnostic: one 64-trajectory handle vs two 32-trajectory handles of the same junction in
one process, their steps enqueued alternately (independent ensembles, separate streams)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def make(N, meta, dyn, baths, B, seed):
    st = N.Stepper(meta["nph"], B, meta["nmd"], meta["dt"], 0, 0, "auto", 0)
    for b in baths:
        W, g = b.gmem_recipe
        st.add_bath_gmem(b.cids, W, g)
    st.set_dyn(dyn)
    rng = np.random.default_rng(seed)
    st.set_state(rng.normal(size=(B, meta["nph"])) * 1e-3, rng.normal(size=(B, meta["nph"])) * 1e-3, 0)
    for i, b in enumerate(baths):
        st.set_history(i, None)
        st.set_noise(i, rng.standard_normal((B, meta["nmd"], b.nc)) * 1e-3)
    return st


def timed(sts, n=512, chunk=int(os.environ.get("CHUNK", "8"))):
    for st in sts:
        st.run(576)
    for st in sts:
        st.sync()
    t0 = time.perf_counter()
    for _ in range(n // chunk):
        for st in sts:
            st.run(chunk)
    for st in sts:
        st.sync()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    from sclmd_amd import _native as N
    from sclmd_amd import synthetic

    dyn, _, baths, meta = synthetic.junction("C3", seed=1234, gmem_device=True)
    out = {"hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}
    st = make(N, meta, dyn, baths, 64, 1)
    out["one_64_us_per_step"] = timed([st])
    st.close()
    a, b = make(N, meta, dyn, baths, 32, 1), make(N, meta, dyn, baths, 32, 2)
    out["two_32_us_per_step"] = timed([a, b])
    a.close()
    b.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
