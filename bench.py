#!/usr/bin/env python3
"""Benchmark of the GLE hot path: trajectory-steps per second on the BASELINE.json workload.

Workload (BASELINE.json metric, configs[2] = SURVEY.md C3): 300-atom chain junction, 2 phonon
baths with nc = 300 coupled DOF each, 1024-step memory kernel, nmd = 4096, fp64, 64 independent
trajectories per GPU (weak scaling: C4 = 8 x 64).  A "step" is one md.vv of every trajectory on
this GPU.  Setup (memory-kernel construction, noise factorisation and generation, H2D) is outside
the timed region.  Before the warm-up an untimed fill (2 x the largest ladder block) brings the
memory-sum ladder to its steady state, so any window of K steps carries K / P blocks of every
level (reported as ladder_window).  Other lines: --config C2 --ntraj 1 (the north-star 1-trajectory
comparison), --config C5 --ntraj 32.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU, RCCL reduce)

Timed window per rank: barrier + device sync, the K steps, device sync (the rank's clock stops
there), then a closing barrier; value uses the MAX of the ranks' window times.

Prints one JSON line (rank 0).  roofline: the dominant kernel (far-field memory-kernel
contraction, cgemm_kernel) timed by its own device timestamps (first workgroup start to last
workgroup end of every launch, s_memrealtime) over a second window of the same K steps, HIP events
on its stream reported beside them; chain_roofline: the per-step chain's launches timed the same
way in a third window; cpu_baseline: the oracle's reference-equivalent numpy step (phonon and
electron baths as the reference builds them, bias terms included) timed on this host for one
trajectory.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X dense FP64 matrix (AMD spec; == FP64 vector peak)
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_info():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model


def blas_info():
    try:
        from threadpoolctl import threadpool_info

        for d in threadpool_info():
            if d.get("user_api") == "blas":
                return "%s %s (%s, %d threads)" % (d.get("internal_api"), d.get("version"),
                                                   d.get("architecture"), d.get("num_threads", 0))
    except Exception:  # pragma: no cover - informational only
        pass
    return "unknown BLAS"


def blas_threads():
    try:
        from threadpoolctl import threadpool_info

        for d in threadpool_info():
            if d.get("user_api") == "blas":
                return int(d.get("num_threads", 1))
    except Exception:  # pragma: no cover
        pass
    return 1


def cpu_baseline(baths_host, dyn, nph, dt, nmd, budget_s=20.0, nsample=5):
    """Time the oracle's reference-shaped step (3 memory passes/step, per-slice matvecs,
    shift-copied history) for ONE trajectory -- the reference runs trajectories one after another
    (md.py:506), so its ensemble throughput equals this single-trajectory rate.  Median of
    `nsample` samples of about budget_s / nsample seconds each, after one warm-up step."""
    from oracle import sclmd_oracle as O

    # baths_host: (kind, cids, kernel, noise, bias terms) -- electron baths keep their bias matrices
    # (ebath.bforce, baths.py:224-255), so a biased C5 bath costs the reference its four matvecs
    bs = [O.Bath(kind, c, k, n, dt, nmd, **extra) for (kind, c, k, n, extra) in baths_host]
    sim = O.GLE(nph, dt, nmd, bs, dyn=dyn)
    rng = np.random.default_rng(0)
    sim.p = rng.normal(size=nph) * 1e-3
    sim.q = rng.normal(size=nph) * 1e-3
    sim.step()  # warm-up
    rates, nsteps = [], 0
    for _ in range(nsample):
        n, t0 = 0, time.perf_counter()
        while True:
            sim.step()
            n += 1
            if time.perf_counter() - t0 > budget_s / nsample:
                break
        rates.append(n / (time.perf_counter() - t0))
        nsteps += n
    return {"value": float(np.median(rates)), "unit": "traj-steps/s", "cores": blas_threads(),
            "kind": "port",
            "sample": "median of %d samples (%d md.vv steps in all) of 1 trajectory of the same junction "
                      "(oracle restatement of sclmd md.vv/phbath.bforce, reference algorithm shape), "
                      "numpy %s + %s, %s" % (nsample, nsteps, np.__version__, blas_info(), cpu_info()),
            "samples": [float(r) for r in rates]}


def cpu_single_pass(baths_host, dyn, nph, dt, nmd, ntraj, budget_s=8.0):
    """Best-effort CPU context number (CPU-baseline plan step 3): the oracle's batched
    step (oracle.GLEBatch: the memory sum once per step as ONE GEMM of the flattened kernel
    [K_1 | ... | K_{ml-1}] with the history window of all ntraj trajectories, BLAS-threaded), timed on
    the same junction and ensemble size as the GPU line.  Context beside the baseline, not the baseline:
    the reference steps one trajectory with three history passes."""
    from oracle import sclmd_oracle as O

    bs = [O.Bath(kind, c, k, n, dt, nmd, **extra) for (kind, c, k, n, extra) in baths_host]
    sim = O.GLEBatch(nph, dt, nmd, bs, dyn, ntr=ntraj)
    rng = np.random.default_rng(0)
    sim.p = rng.normal(size=(nph, ntraj)) * 1e-3
    sim.q = rng.normal(size=(nph, ntraj)) * 1e-3
    sim.step()  # warm-up
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        sim.step()
        n += 1
    el = time.perf_counter() - t0
    return {"value": n * ntraj / el, "unit": "traj-steps/s", "cores": blas_threads(), "kind": "port",
            "sample": "%d steps of a %d-trajectory batch in %.1f s (oracle.GLEBatch: one flattened-kernel GEMM per "
                      "bath per step), numpy %s + %s" % (n, ntraj, el, np.__version__, blas_info())}


METRIC = "GLE steps/sec/GPU, 300-atom junction, 1024-step kernel, 64-traj ensemble"


def loaded_runtime():
    """Paths of the HIP / HSA / RCCL runtimes mapped into this process (torch ships its own copies;
    whichever is loaded first serves every later library that needs the same soname)."""
    out = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                p = line.split()[-1]
                if any(k in os.path.basename(p) for k in ("libamdhip64", "libhsa-runtime64", "librccl")):
                    out.add(p)
    except OSError:
        pass
    return sorted(out)


def refuse_experiment_env():
    """The release library reads no environment; refuse anything that could select the experiment
    build or its switches (some of them skip work and give wrong results)."""
    bad = sorted(k for k in os.environ if k.startswith("GLE_"))
    lib = os.environ.get("SCLMD_AMD_LIB", "")
    if bad or ("_exp" in os.path.basename(lib)):
        raise SystemExit("bench.py: refusing to run with experiment settings %s%s" % (
            bad, (" SCLMD_AMD_LIB=" + lib) if lib else ""))


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_command(nproc, argv, port):
    """torch.distributed.run command line that starts `nproc` ranks of this script (one per GPU) on
    the loopback rendezvous, with the parent's own arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def launch_or_check_world(args, argv):
    """--gpus N > 1 without a torchrun environment: start the N ranks as child processes BEFORE any
    GPU call (the parent never initialises HIP) and return their exit status; under torchrun the
    launcher's WORLD_SIZE must equal --gpus.  Returns None when this process is a rank."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus > 1:
            import subprocess

            env = dict(os.environ)
            env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            cmd = spawn_command(args.gpus, argv, _free_port())
            log("[bench] starting %d ranks: %s" % (args.gpus, " ".join(cmd)))
            return subprocess.call(cmd, env=env)
        return None
    if int(env_world) != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%s (launch one rank per GPU with "
                         "--nproc-per-node equal to --gpus)" % (args.gpus, env_world))
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 512 timed steps = two periods of the largest ladder level (P = 256 at C3)
    ap.add_argument("--steps", type=int, default=512)
    ap.add_argument("--warmup", type=int, default=64)
    ap.add_argument("--ntraj", type=int, default=64, help="trajectories per GPU")
    ap.add_argument("--config", default="C3", choices=["C2", "C3", "C5"])
    ap.add_argument("--block-len", type=int, default=0)
    ap.add_argument("--max-block", type=int, default=0)
    ap.add_argument("--far-mode", default="auto", choices=["auto", "direct", "spectral"])
    ap.add_argument("--gmem", default="device", choices=["device", "host"],
                    help="memory-kernel construction (phbath.gmem) on the device or with numpy")
    ap.add_argument("--noise", default="device", choices=["device", "white"],
                    help="device: coloured noise from the bath spectra (factorised on the host, drawn "
                         "and filtered on the device); white: seeded N(0, 1e-3^2) realisations assigned "
                         "to bath.noise (throughput runs only; the step does the same work)")
    ap.add_argument("--fill", type=int, default=-1,
                    help="untimed steps before the warm-up that bring the memory-sum ladder to its steady "
                         "state (history older than the largest level's window); -1 = 2 x the largest "
                         "block length, then a scan of K-step windows over the largest level's period "
                         "and the timed window at the phase closest to the mean")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo only to "
                         "rehearse the multi-rank path, e.g. with --same-device on a one-GPU box)")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on device 0 (rehearsal of the N > 1 control flow on one GPU)")
    ap.add_argument("--early-collective", action="store_true",
                    help="one collective right after the process group is joined, before the stepper exists "
                         "(RCCL's streams then take their hardware queues first; rehearsal of a host program "
                         "that communicates before it builds the stepper)")
    ap.add_argument("--stream-noise", action="store_true",
                    help="generate the coloured noise through the streamed-factor path whatever the bath size "
                         "(the C5 path; rehearses the node-shared factorisation at small configs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--single-pass-budget", type=float, default=8.0,
                    help="seconds of the best-effort batched CPU context number (0: skip)")
    ap.add_argument("--traffic-json", default="",
                    help="PMC-derived HBM bytes per dominant-kernel launch (from rocprofv3 --pmc passes); "
                         "default: profiles/traffic_<config>_<ntraj>.json if present, else "
                         "profiles/traffic_latest.json (used only when its config / ntraj / plan match)")
    args = ap.parse_args()
    refuse_experiment_env()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    rc = launch_or_check_world(args, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    if not args.traffic_json:
        per = os.path.join(ROOT, "profiles", "traffic_%s_%d.json" % (args.config, args.ntraj))
        args.traffic_json = per if os.path.exists(per) else os.path.join(ROOT, "profiles", "traffic_latest.json")

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # Under a launcher (WORLD_SIZE set, world 1 included) the rank joins the process group, so a
    # world-1 `torchrun --nproc-per-node 1` run has RCCL's communicator and streams beside the
    # stepper's (the multi-GPU path rehearsed on one GPU); a plain `python bench.py` has no group.
    if "WORLD_SIZE" in os.environ:
        import torch
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.same_device:
            local_rank = 0
        elif torch.cuda.device_count() < world:
            raise SystemExit("bench.py: %d ranks but %d visible GPUs (one rank per GPU; --same-device "
                             "rehearses the multi-rank path on one)" % (world, torch.cuda.device_count()))
        torch.cuda.set_device(local_rank)
        dist.init_process_group(args.dist_backend)
        if dist.get_world_size() != args.gpus:
            raise SystemExit("bench.py: process group has %d ranks, --gpus %d" % (dist.get_world_size(), args.gpus))
        world, rank = dist.get_world_size(), dist.get_rank()
        if args.early_collective:
            dist.barrier()

    from sclmd_amd import md as MD
    from sclmd_amd import synthetic

    t_setup = time.perf_counter()
    dyn, axyz, baths, meta = synthetic.junction(args.config, seed=1234, gmem_device=args.gmem == "device")
    m = MD.md(meta["dt"], meta["nmd"], meta["T"], axyz=axyz, dyn=dyn, ntraj=args.ntraj,
              seed=1000, traj_offset=rank * args.ntraj, device=local_rank,
              noise_mode="device", block_len=args.block_len, far_mode=args.far_mode,
              max_block=args.max_block, verbose=False)
    log("[bench] rank %d system built (%.1fs)" % (rank, time.perf_counter() - t_setup))
    for b in baths:
        m.AddBath(b)
    if args.stream_noise:
        m.noise_stream_bytes = 0
    m.initialise()
    m.ResetHis()
    log("[bench] rank %d state initialised (%.1fs)" % (rank, time.perf_counter() - t_setup))
    noise_s = 0.0
    if args.noise == "white":
        rng = np.random.default_rng(4321 + rank)
        for b in baths:
            b.noise = rng.standard_normal((args.ntraj, meta["nmd"], b.nc)) * 1e-3
    else:
        t_noise = time.perf_counter()
        for i in range(len(baths)):
            tn = time.perf_counter()
            m.gen_noise(i, 0)
            log("[bench] rank %d noise of bath %d (%s, nc %d): %.1fs" % (rank, i, baths[i].kind, baths[i].nc,
                                                                      time.perf_counter() - tn))
        noise_s = time.perf_counter() - t_noise
    st = m._ensure_device()
    tp = time.perf_counter()
    m.steps(0)  # uploads assigned noise
    st.sync()
    log("[bench] rank %d plan / first prime: %.1fs" % (rank, time.perf_counter() - tp))
    setup_s = time.perf_counter() - t_setup
    plan = st.plan_info()
    detail = st.plan_detail()
    log("[bench] rank %d setup %.1fs plan %s %s" % (rank, setup_s, plan, detail))
    # per-rank setup: wall time, noise phase and the noise factorisations this rank computed (the
    # ranks of a node split them, noise.NodeShare: their sum is one rank's count alone)
    row = np.zeros((world, 3))
    row[rank] = [setup_s, noise_s, float(getattr(m, "noise_factorisations", -1))]
    setup_ranks = m._allreduce(row) if world > 1 else row

    def barrier():
        if dist is not None:
            dist.barrier()

    # RCCL sets a communicator up lazily: its first collectives cost up to ~2 ms each (profiles/r05,
    # rt_nccl*), so two untimed ones go before the ladder fill
    barrier()
    barrier()

    levels = st.profile_levels()
    ptop = max([P for P, _ in levels] + [1])
    t_now = st.get_state()[2]
    t_fill = time.perf_counter()
    phase = None
    fill = 2 * ptop if args.fill < 0 else args.fill
    m.steps(fill)
    nscan = ptop // math.gcd(args.steps, ptop)
    if args.fill < 0 and levels and nscan > 1:
        # The ladder's background work within a short window depends on where the window falls in
        # the largest level's period (blocks start at multiples of P, their pieces follow), so a
        # K-step window is timed at every phase it can take (consecutive untimed windows, each
        # bracketed like the timed one), and the timed window starts at the phase whose time is
        # closest to the mean over all phases, i.e. a window representative of the steady state.
        nscan = min(nscan, 128)
        times = []
        for _ in range(nscan):
            tp = (t_now + fill) % ptop
            st.sync()
            ts = time.perf_counter()
            m.steps(args.steps)
            st.sync()
            times.append((tp, (time.perf_counter() - ts) / args.steps * 1e3))
            fill += args.steps
        mean = float(np.mean([x for _, x in times]))
        phi, tphi = min(times, key=lambda pt: abs(pt[1] - mean))
        adv = (phi - args.warmup - (t_now + fill)) % ptop
        m.steps(adv)
        fill += adv
        ms = [x for _, x in times]
        phase = {"t_mod_ptop": int(phi), "ptop": int(ptop), "phases_scanned": len(times),
                 "scan_ms_per_step": {"mean": round(mean, 5), "min": round(min(ms), 5), "max": round(max(ms), 5),
                                      "chosen": round(tphi, 5)}}
    st.sync()
    log("[bench] rank %d ladder fill %d steps (%.2fs)" % (rank, fill, time.perf_counter() - t_fill))
    m.steps(args.warmup)
    st.sync()
    st.profile(True, events=False)  # ladder block counts of the timed window
    # The window: barrier + device sync, K steps, device sync; each rank's clock stops when its
    # device has finished the K steps, the closing barrier follows, and el is the MAX over ranks
    # (below), i.e. the time until the last rank's K steps are done.  The closing barrier itself is
    # not timed: an RCCL barrier costs 0.1-0.4 ms (profiles/r05/rt_*.json), 10-40 % of a 20-step
    # window, and it is not work of the K steps.
    barrier()
    st.sync()
    t0 = time.perf_counter()
    m.steps(args.steps)
    t_enq = time.perf_counter() - t0
    st.sync()
    el = time.perf_counter() - t0
    barrier()
    log("[bench] rank %d host enqueue %.3f ms of %.3f ms timed" % (rank, t_enq * 1e3, el * 1e3))
    window_levels = st.profile_levels()
    # roofline: HIP events around every launch of the dominant kernel over a second window of the
    # same K steps right after the timed one (same steady state, same piece schedule phase); the
    # events add launch-queue packets (1-6 % per step), so the headline window runs without them.
    # Fused schedule: the far-field GEMMs ride in the chain launches, which the third window times.
    if not detail["far_fused"]:
        st.profile(True, events=True)
        m.steps(args.steps)
        st.sync()
        prof = st.profile_read()
    else:
        prof = {"launches": 0}
    # the chain's own per-workgroup stamps in a third window of the same K steps (apart from the
    # far-field timing, whose launches the chain stamps would otherwise share the window with)
    st.profile(True, events=False, chain=True)
    m.steps(args.steps)
    st.sync()
    pch = st.profile_read()
    prof.update({k: pch[k] for k in ("chain_launches", "chain_ms", "chain_flops")})
    st.profile(False)
    # one reduce of the time-averaged current statistics (the ensemble output)
    sums = m._reduce(st.current_sums())
    if dist is not None:
        import torch

        tt = torch.tensor([el], dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())

    value = world * args.ntraj * args.steps / el
    ms_per_step = el / args.steps * 1e3
    res = {
        "metric": METRIC,
        "value": value,
        "unit": "traj-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded chain junction, device gmem kernels, %s)" % (
            "device Philox coloured noise" if args.noise == "device" else "injected white noise, throughput only"),
        "config": {"workload": "%s: %d-atom chain junction, %d baths nc=%s, ml=%d, nmd=%d, "
                               "%d traj/GPU" % (args.config, meta["natom"], len(baths), meta["nc"],
                                                meta["ml"], meta["nmd"], args.ntraj),
                   "ntraj_per_gpu": args.ntraj, "ntraj_total": world * args.ntraj,
                   "block_len": plan["block_len"], "far_mode": plan["far_mode"],
                   "far_schedule": "fused" if detail["far_fused"] else "background",
                   "plan_class": detail["plan_class"],
                   "chain_launches_per_step": 1 if detail.get("composed_step") else (
                       2 + (1 if detail.get("fpot_launch") else 0)),
                   "parallelism": "ensemble-dp%d" % world},
        "value_per_gpu": value / world,
        "runtime_libs": loaded_runtime(),
        "setup_s": setup_s,
        "setup_ranks": [{"rank": r, "setup_s": round(float(v[0]), 3), "noise_s": round(float(v[1]), 3),
                         "factorisations": (int(v[2]) if v[2] >= 0 else None)}
                        for r, v in enumerate(np.asarray(setup_ranks).reshape(world, 3))],
        "fill_steps": fill,
        "window_t0": int(t_now + fill + args.warmup),
        "window_phase": phase,
        # per ladder level: blocks issued in the timed window vs the steady-state share K / P
        "ladder_window": [{"P": P, "blocks": round(bl, 3), "steady": round(args.steps / P, 3)}
                          for P, bl in window_levels],
    }
    # whole-step roofline: the algorithm's own work per step (SURVEY.md 8d conventions, gle_step_work)
    fl_step, by_step = st.step_work()
    res["step_roofline"] = {
        "flops_per_step": fl_step, "bytes_per_step": by_step,
        "achieved_tflops": fl_step / (ms_per_step * 1e-3) / 1e12,
        "frac_mfma": fl_step / (ms_per_step * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS,
        "achieved_gbs": by_step / (ms_per_step * 1e-3) / 1e9,
        "frac_hbm": by_step / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
    }
    if prof["launches"] > 0:
        # kernel duration of each launch from the device's own timestamps (first workgroup start to
        # last workgroup end, what a kernel trace reports); the HIP-event average also counts each
        # launch's wait for free CUs on its stream and is reported beside it
        avg_ev = prof["ms"] / prof["launches"]
        avg_ms = prof["ms_device"] / prof["launches_device"] if prof["launches_device"] == prof["launches"] else avg_ev
        fl = prof["flops"] / prof["launches"]
        by = prof["bytes"] / prof["launches"]
        ai = fl / max(by, 1.0)
        ridge = FP64_MFMA_PEAK_TFLOPS * 1e12 / (HBM_PEAK_GBS * 1e9)
        if ai >= ridge:
            roof = {"bound": "mfma", "achieved": fl / (avg_ms * 1e-3) / 1e12, "peak": FP64_MFMA_PEAK_TFLOPS,
                    "unit": "TFLOP/s"}
        else:
            roof = {"bound": "hbm", "achieved": by / (avg_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s"}
        roof["frac"] = roof["achieved"] / roof["peak"]
        roof["traffic"] = None
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if (tj.get("config") == args.config and tj.get("ntraj") == args.ntraj
                    and tj.get("far_mode") == plan["far_mode"]):
                roof["traffic"] = tj.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            pass
        if plan["far_mode"] == "spectral":
            kname = ("cgemm_kernel (far field: per-frequency Gauss 3-multiplication GEMMs of the "
                     "spectral ladder levels)")
        else:
            kname = "contract_kernel (far field: direct ladder-level memory-kernel contraction)"
        roof.update({"kernel": kname, "window": "second window of the same %d steps" % args.steps,
                     "launches": prof["launches"], "avg_launch_ms": avg_ms, "avg_launch_ms_hip_events": avg_ev,
                     "timing": "device timestamps" if prof["launches_device"] == prof["launches"] else "HIP events",
                     "algorithmic_flops_per_launch": fl, "algorithmic_bytes_per_launch": by})
        res["roofline"] = roof
    if detail["far_fused"] and prof.get("chain_launches", 0) > 0:
        # fused schedule: every launch of the step is the chain kernel (md.vv stages plus the
        # spectral levels' far-field GEMM items), timed by its own per-workgroup device stamps in the
        # third window; algorithmic flops = the chain products + the items' share of their blocks
        cms = prof["chain_ms"]
        nl = prof["chain_launches"]
        roof = {"bound": "mfma", "achieved": prof["chain_flops"] / (cms * 1e-3) / 1e12, "peak": FP64_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s"}
        roof["frac"] = roof["achieved"] / roof["peak"]
        roof["traffic"] = None
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if (tj.get("config") == args.config and tj.get("ntraj") == args.ntraj
                    and tj.get("kernel", "").startswith("chain_kernel") and tj.get("far_schedule") == "fused"):
                roof["traffic"] = tj.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            pass
        roof.update({"kernel": "chain_kernel (fused: md.vv stage A / velocity stage + far-field GEMM items of the "
                               "spectral ladder levels)",
                     "window": "third window of the same %d steps" % args.steps, "launches": nl,
                     "avg_launch_ms": cms / nl, "us_per_step": cms / args.steps * 1e3,
                     "timing": "device timestamps (per-workgroup stores)",
                     "algorithmic_flops_per_launch": prof["chain_flops"] / nl})
        res["roofline"] = roof
    if prof.get("chain_launches", 0) > 0 and not detail["far_fused"]:
        # the per-step chain (md.vv stages, the step's critical path) in the same window, timed by
        # its own device timestamps: algorithmic flops of its products / its kernel durations;
        # us_per_step = chain kernel time per step (beside the far field, so > its time alone)
        cms = prof["chain_ms"]
        _, cby = st.chain_work()  # algorithmic bytes of one step's chain launches (every entry once)
        tf = prof["chain_flops"] / (cms * 1e-3) / 1e12
        gbs = cby * args.steps / (cms * 1e-3) / 1e9
        # one-trajectory composed plans run the chain's products on the VALU (one column: chain stage
        # 5, a GEMV): their rate is priced on bytes, the MFMA-tiled plans' on the fp64 matrix peak
        gemv = bool(detail.get("composed_step")) and args.ntraj == 1
        res["chain_roofline"] = {
            "kernel": "chain_kernel (per-step md.vv: %s)" % (
                ("one composed launch, one-column VALU products (GEMV)" if gemv else "one composed launch")
                if detail.get("composed_step") else "stage A and the fused velocity stage"),
            "bound": "hbm" if gemv else "mfma",
            "achieved": gbs if gemv else tf,
            "peak": HBM_PEAK_GBS if gemv else FP64_MFMA_PEAK_TFLOPS,
            "unit": "GB/s" if gemv else "TFLOP/s",
            "frac": gbs / HBM_PEAK_GBS if gemv else tf / FP64_MFMA_PEAK_TFLOPS,
            "achieved_tflops": tf, "frac_mfma": tf / FP64_MFMA_PEAK_TFLOPS,
            "achieved_gbs": gbs, "frac_hbm": gbs / HBM_PEAK_GBS,
            "launches": prof["chain_launches"], "us_per_step": cms / args.steps * 1e3,
            "algorithmic_flops_per_step": prof["chain_flops"] / args.steps,
            "algorithmic_bytes_per_step": cby,
            "timing": "device timestamps (per-workgroup stores)",
            "window": "third window of the same %d steps" % args.steps}
    # The reduce runs (it is the ensemble's one collective), but its result is not reported: over a
    # bench window the run is partly filled and not in steady state, so the mean current is neither
    # md.Run's per-run kappa (md.py:657-664) nor tools.calTC's estimate (tools.py:191-201).
    res["ensemble_reduce"] = {"doubles": int(sums.size), "backend": (args.dist_backend if dist is not None else "none"),
                              "world": world}

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        noise = [st.get_noise(i)[0] for i in range(len(baths))]
        bh = []
        for i, b in enumerate(baths):
            if b.kind == "ebath":  # the host kernel (efric, ml = 1): the device copy has zeta2 folded in
                bh.append(("e", b.cids, b.kernel, noise[i],
                           dict(bias=b.bias, exim=b.exim, zeta1=b.zeta1, zeta2=b.zeta2)))
            else:
                bh.append(("ph", b.cids, st.get_kernel(i), noise[i], {}))
        res["cpu_baseline"] = cpu_baseline(bh, m.dyn, meta["nph"], meta["dt"], meta["nmd"], args.cpu_budget)
        res["speedup_vs_cpu_baseline"] = value / res["cpu_baseline"]["value"]
        if args.single_pass_budget > 0:
            res["cpu_baseline"]["single_pass"] = cpu_single_pass(bh, m.dyn, meta["nph"], meta["dt"], meta["nmd"],
                                                                 args.ntraj, args.single_pass_budget)
    if rank == 0:
        print(json.dumps(res), flush=True)
    m.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
