#!/usr/bin/env python3
"""Timing experiments on the GPU box (not the bench): C3-like junction, white noise (same step work
as coloured noise), ladder fill, a short window (the driver's 20 steps after 5) and a long window.
The library is picked with SCLMD_AMD_LIB (experiment builds read GLE_* switches).  --variants runs
several GLE_* settings interleaved over --rounds in ONE process (one box, A/B/A/B), because
boxes differ by several percent; prints one JSON line per measurement.

    SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so python scripts/exp_time.py \\
        --variants "GLE_PIECE_SLACK=1;GLE_PIECE_SLACK=0" --rounds 3
"""
import argparse
import json
import os
import re
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dist_barrier(args):
    if args.dist != "none":
        import torch.distributed as dist

        dist.barrier()


def dist_init(args):
    """A world-1 torch.distributed nccl (RCCL) group with one collective: torch's stream pools and
    RCCL's streams exist from then on (bench.py's multi-rank path)."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % args.port, rank=0, world_size=1)
    dist.barrier()


def measure(args, meta, dyn, baths):
    from sclmd_amd import _native as N

    B = args.ntraj
    if args.dist == "before":
        dist_init(args)
    st = N.Stepper(meta["nph"], B, meta["nmd"], meta["dt"], 0, int(os.environ.get("EXP_BLOCK_LEN", "0")), "auto",
                   int(os.environ.get("EXP_MAX_BLOCK", "0")))
    try:
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
        ptop = max([P for P, _ in st.profile_levels()] + [1])
        if args.dist == "after":
            dist_init(args)
        st.run(2 * ptop + 5)
        st.sync()
        if args.profile:
            st.profile(True)
        elif args.chainprof:
            st.profile(True, events=False, chain=True)
        dist_barrier(args)
        st.sync()
        t0 = time.perf_counter()
        st.run(args.short)
        st.sync()
        dist_barrier(args)
        el_short = time.perf_counter() - t0
        # the same window started on a piece-slot boundary (t = 0 mod P0)
        st.run((-(2 * ptop + 5 + args.short)) % st.plan_info()["block_len"])
        st.sync()
        t0 = time.perf_counter()
        st.run(args.short)
        st.sync()
        el_aligned = time.perf_counter() - t0
        st.run(64)
        st.sync()
        dist_barrier(args)
        st.sync()
        t0 = time.perf_counter()
        st.run(args.steps)
        st.sync()
        dist_barrier(args)
        el = time.perf_counter() - t0
        prof = st.profile_read() if (args.profile or args.chainprof) else None
        if args.profile or args.chainprof:
            st.profile(False)
        reps = []
        for _ in range(args.short_reps):  # bench-like short windows: sync, K steps, sync
            st.run(37)
            st.sync()
            dist_barrier(args)
            st.sync()
            t0 = time.perf_counter()
            st.run(args.short)
            st.sync()
            dist_barrier(args)
            reps.append(round((time.perf_counter() - t0) / args.short * 1e3, 5))
        scan = []
        if args.phase_scan:  # bench.py's scan: consecutive sync-bracketed K-step windows over the period
            K = args.phase_scan
            for _ in range(max(1, ptop // K)):
                t_now = st.get_state()[2]
                st.sync()
                t0 = time.perf_counter()
                st.run(K)
                st.sync()
                scan.append((int(t_now % ptop), round((time.perf_counter() - t0) / K * 1e3, 5)))
        wins = {}
        for K in [int(x) for x in args.windows.split(",") if x]:  # window-length sweep: t(K) = a + b K
            ts = []
            for _ in range(args.window_reps):
                st.run(29)
                st.sync()
                t0 = time.perf_counter()
                st.run(K)
                st.sync()
                ts.append((time.perf_counter() - t0) * 1e3)
            wins[K] = round(float(np.median(ts)), 4)
        p, q, _ = st.get_state()
    finally:
        st.close()
    extra = {}
    if prof and prof.get("chain_launches"):
        # chain kernel time per step (launch spans, device stamps) over every profiled step
        nst = args.short * 2 + 64 + args.steps
        extra["chain_us_per_step"] = prof["chain_ms"] * 1e3 / max(1, prof["chain_launches"] / 2)
    if prof and prof.get("launches"):
        ms = prof.get("ms_device") or prof["ms"]
        extra = {"cgemm_launches": prof["launches"], "cgemm_avg_us": ms / prof["launches"] * 1e3,
                 "cgemm_tflops": prof["flops"] / (ms * 1e-3) / 1e12}
    return {**extra, "ms_per_step": el / args.steps * 1e3, "short_ms_per_step": el_short / max(args.short, 1) * 1e3,
            "aligned_short_ms_per_step": el_aligned / max(args.short, 1) * 1e3, "short_reps_ms": reps,
            "traj_steps_per_s": B * args.steps / el, "window_ms": wins, "phase_scan": scan, "finite": bool(np.isfinite(p).all() and np.isfinite(q).all())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--ntraj", type=int, default=64)
    ap.add_argument("--steps", type=int, default=512)
    ap.add_argument("--short", type=int, default=20, help="short window (the driver's 20 after 5)")
    ap.add_argument("--variants", default="", help="';'-separated variants of ','-separated GLE_X=V")
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--tag", default="")
    ap.add_argument("--short-reps", type=int, default=0, help="extra short windows at drifting phases")
    ap.add_argument("--profile", type=int, default=0, help="HIP-event timing of the far-field launches on")
    ap.add_argument("--chainprof", type=int, default=0, help="device stamps of the chain launches on")
    ap.add_argument("--windows", default="", help="comma-separated window lengths: median ms per window")
    ap.add_argument("--window-reps", type=int, default=9)
    ap.add_argument("--dist", default="none", choices=["none", "before", "after"],
                    help="world-1 nccl process group joined before / after the stepper is created, windows "
                         "bracketed by its barrier (bench.py's multi-rank timing)")
    ap.add_argument("--port", type=int, default=29701)
    ap.add_argument("--phase-scan", type=int, default=0, help="K: K-step windows over the largest period")
    args = ap.parse_args()
    if args.dist != "none":
        # torch first: the library then binds to torch's HIP runtime (one runtime per process, as in
        # bench.py's multi-rank path; the other order loads two runtimes and torch's cannot start)
        import torch  # noqa: F401
    from sclmd_amd import synthetic

    dyn, _, baths, meta = synthetic.junction(args.config, seed=1234, gmem_device=True)
    variants = [v for v in args.variants.split(";")] if args.variants else [""]
    if len(variants) > 1 and any("GLE_BG_SAMEPRIO" in v for v in variants):
        # once a handle has created its background streams at the main stream's priority, every
        # later handle of the process with mixed priorities ran at ~115 instead of 49 us/step (HIP's
        # hardware-queue reuse, r04 `profiles/r04/sched_priority_mixing_trap_c3.jsonl`)
        sys.exit("GLE_BG_SAMEPRIO changes the process's hardware-queue mapping: time it in a process of its own")
    base = {k: v for k, v in os.environ.items() if k.startswith("GLE_") or k.startswith("EXP_")}
    for r in range(args.rounds):
        for v in variants:
            for k in [k for k in os.environ if k.startswith("GLE_") or k.startswith("EXP_")]:
                del os.environ[k]
            env = dict(base)
            for kv in filter(None, re.split(r",(?=(?:GLE_|EXP_))", v)):
                k, val = kv.split("=", 1)
                env[k] = val
            os.environ.update(env)
            out = {"tag": args.tag, "profile": args.profile, "variant": v, "round": r,
                   "lib": os.path.basename(os.environ.get("SCLMD_AMD_LIB", "libhipgle.so")), "env": env,
                   "config": args.config, "ntraj": args.ntraj, "steps": args.steps}
            out.update(measure(args, meta, dyn, baths))
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
