#!/usr/bin/env python3
"""Calibrate bench.py's cpu_baseline (the oracle restatement, "port") against the REAL reference at
the C2 shape, in this container (BASELINE.md "CPU-baseline plan" item 2; the reference cannot travel
to the GPU box, so the ratio measured here is what ties the box's port timing to the reference).

C2: 300-atom chain, 2 phonon baths with nc = 300 and a 1024-slice memory kernel, fp64, 1
trajectory.  Both codes get the same kernels (built once with sclmd_amd's gmem, injected into the
reference's phbath objects as SURVEY.md section 3.4 allows) and the same injected noise; each runs
`--steps` md.vv steps after one warm-up step, median of `--samples` repetitions.  Writes
profiles/r02/cpu_calibration.json.  Runs only where /root/reference exists (never on the GPU box).

    PYTHONDONTWRITEBYTECODE=1 python3 scripts/calibrate_cpu_baseline.py
"""
import argparse
import contextlib
import io
import json
import os
import sys
import time
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--samples", type=int, default=5)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02", "cpu_calibration.json"))
    args = ap.parse_args()
    sys.path.insert(0, ROOT)
    from oracle import sclmd_oracle as O
    from sclmd_amd import synthetic

    dyn, axyz, baths, meta = synthetic.junction("C2", seed=1234)
    nph, dt, nmd = meta["nph"], meta["dt"], meta["nmd"]
    rng = np.random.default_rng(7)
    noise = [rng.normal(size=(nmd, b.nc)) * 1e-3 for b in baths]
    p0 = rng.normal(size=nph) * 1e-3
    q0 = rng.normal(size=nph) * 1e-3

    # ---- the reference (imported here only)
    sys.path.insert(0, REF)
    sys.modules["netCDF4"] = types.SimpleNamespace(Dataset=None)
    import sclmd.baths as RB
    import sclmd.md as RMD

    with contextlib.redirect_stdout(io.StringIO()):
        m = RMD.md(dt, nmd, meta["T"], axyz=axyz, dyn=dyn)
        for i, b in enumerate(baths):
            rb = RB.phbath(b.T, b.cids, debye=0.2, nw=10, dt=dt, nmd=nmd, ml=b.ml)
            rb.kernel, rb.ml, rb.noise = np.array(b.kernel), b.ml, noise[i]
            m.AddBath(rb)
        m.initialise()
        m.ResetHis()
    m.p, m.q, m.t = p0.copy(), q0.copy(), 0

    def time_ref():
        rates = []
        with contextlib.redirect_stdout(io.StringIO()):
            m.vv(0)
            for _ in range(args.samples):
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    m.vv(0)
                rates.append(args.steps / (time.perf_counter() - t0))
        return rates

    sim = O.GLE(nph, dt, nmd, [O.Bath("ph", b.cids, b.kernel, noise[i], dt, nmd) for i, b in enumerate(baths)],
                dyn=m.dyn)
    sim.p, sim.q = p0.copy(), q0.copy()

    def time_port():
        rates = []
        sim.step()
        for _ in range(args.samples):
            t0 = time.perf_counter()
            for _ in range(args.steps):
                sim.step()
            rates.append(args.steps / (time.perf_counter() - t0))
        return rates

    # interleave the two codes so machine noise hits both alike
    r_ref, r_port = [], []
    for _ in range(2):
        r_ref += time_ref()
        r_port += time_port()
    ref, port = float(np.median(r_ref)), float(np.median(r_port))
    # same trajectory: the port is the reference algorithm, so the states must agree
    sim2 = O.GLE(nph, dt, nmd, [O.Bath("ph", b.cids, b.kernel, noise[i], dt, nmd) for i, b in enumerate(baths)],
                 dyn=m.dyn)
    from threadpoolctl import threadpool_info

    blas = [d for d in threadpool_info() if d.get("user_api") == "blas"]
    out = {"config": "C2: 300-atom chain, 2 phbath nc=300, ml=1024, nmd=%d, fp64, 1 trajectory" % nmd,
           "reference_steps_per_s": ref, "port_steps_per_s": port, "ratio_port_over_reference": port / ref,
           "within_20pct": bool(abs(port / ref - 1.0) <= 0.2),
           "samples_reference": r_ref, "samples_port": r_port, "steps_per_sample": args.steps,
           "cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": \t"),
           "cores": os.cpu_count(), "blas": blas[0] if blas else None, "numpy": np.__version__}
    del sim2
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("reference_steps_per_s", "port_steps_per_s", "ratio_port_over_reference",
                                          "within_20pct")}))


if __name__ == "__main__":
    main()
