#!/usr/bin/env python3
"""Timing experiments on the GPU box (not the bench): one process, C3-like junction, white noise
(same step work as coloured noise), ladder fill, then `--steps` timed steps.  The library is picked
with SCLMD_AMD_LIB (experiment builds read GLE_* switches); prints one JSON line with ms/step.

    SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so GLE_CHAIN_NW=4,16,4 python scripts/exp_time.py
"""
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
    ap.add_argument("--config", default="C3")
    ap.add_argument("--ntraj", type=int, default=64)
    ap.add_argument("--steps", type=int, default=512)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    from sclmd_amd import _native as N
    from sclmd_amd import synthetic

    dyn, _, baths, meta = synthetic.junction(args.config, seed=1234, gmem_device=True)
    B = args.ntraj
    st = N.Stepper(meta["nph"], B, meta["nmd"], meta["dt"], 0, 0, "auto", 0)
    for b in baths:
        if b.kind == "ebath":
            st.add_bath(N.GLE_BATH_ELECTRON, b.cids, b.kernel, b.bias, b.exim, b.zeta1, b.zeta2)
        else:
            W, g = b.gmem_recipe
            st.add_bath_gmem(b.cids, W, g)
    st.set_dyn(dyn)
    rng = np.random.default_rng(1)
    st.set_state(rng.normal(size=(B, meta["nph"])) * 1e-3, rng.normal(size=(B, meta["nph"])) * 1e-3, 0)
    for i, b in enumerate(baths):
        st.set_history(i, None)
        st.set_noise(i, rng.standard_normal((B, meta["nmd"], b.nc)) * 1e-3)
    levels = st.profile_levels()
    ptop = max([P for P, _ in levels] + [1])
    st.run(2 * ptop + 64)
    st.sync()
    t0 = time.perf_counter()
    st.run(args.steps)
    st.sync()
    el = time.perf_counter() - t0
    p, q, t = st.get_state()
    st.close()
    out = {"tag": args.tag, "lib": os.path.basename(os.environ.get("SCLMD_AMD_LIB", "libhipgle.so")),
           "env": {k: v for k, v in os.environ.items() if k.startswith("GLE_")},
           "config": args.config, "ntraj": B, "steps": args.steps, "ms_per_step": el / args.steps * 1e3,
           "traj_steps_per_s": B * args.steps / el, "finite": bool(np.isfinite(p).all() and np.isfinite(q).all())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
