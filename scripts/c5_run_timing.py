#!/usr/bin/env python3
"""End-to-end md.Run wall time per run at C5 (one GPU's share: 1000-atom junction, 32 trajectories,
ml 4096, nmd 8192, coloured noise streamed), split into its parts: per-run noise generation
(md.gen_noise: factorisation on the first run, the cached factors afterwards), stepping, and the
MD{j}.nc checkpoint (dump, and the previous run's file read back at the next run's start, md.py:506-567).

    python scripts/c5_run_timing.py --runs 3 [--workdir /tmp/c5run]

Prints one JSON line."""
import argparse
import collections
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--ntraj", type=int, default=32)
    ap.add_argument("--nmd", type=int, default=0, help="override nmd (0: the config's 8192)")
    ap.add_argument("--workdir", default="")
    args = ap.parse_args()
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic

    wd = args.workdir or tempfile.mkdtemp(prefix="c5run")
    os.makedirs(wd, exist_ok=True)
    cwd = os.getcwd()
    os.chdir(wd)
    t_all = time.perf_counter()
    dyn, axyz, baths, meta = synthetic.junction("C5", seed=1234, gmem_device=True, nmd=args.nmd or None)
    m = MD.md(meta["dt"], meta["nmd"], meta["T"], axyz=axyz, dyn=dyn, ntraj=args.ntraj, seed=1000, nstart=0,
              nstop=args.runs, noise_mode="device", verbose=False)
    for b in baths:
        m.AddBath(b)
    m.RemoveNC(True)
    parts = collections.defaultdict(lambda: collections.defaultdict(float))
    cur = {"run": -1}

    def log(*a):
        print("[c5run %.1fs]" % (time.perf_counter() - t_all), *a, file=sys.stderr, flush=True)

    def timed(name, fn):
        def w(*a, **k):
            t0 = time.perf_counter()
            try:
                return fn(*a, **k)
            finally:
                if name == "dump":
                    m._st.sync()
                    phases()
                parts[cur["run"]][name] += time.perf_counter() - t0
                log("run %d %s %.2fs" % (cur["run"], name, time.perf_counter() - t0))
        return w

    orig_resume = m._resume

    def resume(j):
        cur["run"] = j
        t0 = time.perf_counter()
        r = orig_resume(j)
        parts[j]["resume_incl_noise"] += time.perf_counter() - t0
        return r

    m._resume = resume
    m.gen_noise = timed("noise", m.gen_noise)
    orig_steps = m.steps

    def steps(n):
        t0 = time.perf_counter()
        orig_steps(n)
        m._st.sync()
        parts[cur["run"]]["steps"] += time.perf_counter() - t0
        parts[cur["run"]]["nsteps"] += n
        log("run %d %d steps %.2fs" % (cur["run"], n, time.perf_counter() - t0))

    m.steps = steps
    m.dump = timed("dump", m.dump)
    seen = {}

    def phases():  # md.phase_times accumulated since the last call, per run
        pt = dict(getattr(m, "phase_times", {}))
        for k, v in pt.items():
            d = v - seen.get(k, 0.0)
            if d:
                parts[cur["run"]]["phase_" + k] += d
        seen.update(pt)

    t_run = time.perf_counter()
    m.Run()
    t_end = time.perf_counter()
    phases()
    kappa = [list(map(float, k)) for k in m.kappa_runs]
    m.close()
    os.chdir(cwd)
    if not args.workdir:
        shutil.rmtree(wd, ignore_errors=True)
    runs = {}
    for j, d in sorted(parts.items()):
        if j < 0:
            continue
        d = dict(d)
        d["resume_other"] = d.pop("resume_incl_noise", 0.0) - d.get("noise", 0.0)
        d["total"] = d["resume_other"] + d.get("noise", 0.0) + d.get("steps", 0.0) + d.get("dump", 0.0)
        d["traj_steps_per_s_stepping"] = args.ntraj * d.get("nsteps", 0) / max(d.get("steps", 1e-9), 1e-9)
        runs[j] = {k: round(v, 3) for k, v in d.items()}
    print(json.dumps({"config": "C5", "ntraj": args.ntraj, "nmd": meta["nmd"], "runs": runs,
                      "setup_before_run_s": round(t_run - t_all, 2), "run_total_s": round(t_end - t_run, 2),
                      "kappa_nW": kappa}), flush=True)


if __name__ == "__main__":
    main()
