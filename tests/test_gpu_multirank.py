"""The multi-rank ensemble through the product stepper, rehearsed on one GPU: every rank
on device 0, torch.distributed over gloo (the 8-GPU node's nccl/RCCL path differs only in the
backend of the one per-run all-reduce, ensemble.allreduce_sums).

* md.Run on two ranks of 4 trajectories each (traj_offset = rank * 4) through the HIP stepper gives
  the per-run ensemble heat current (kappa) of one rank with all 8 trajectories, and the same final
  states (trajectory g's initial state and device noise are keyed by its global index);
* bench.py --gpus 2 (no torchrun environment) starts its two ranks itself and reports the live
  group's size and the whole ensemble.

Replaces the reference's sequential ensemble (md.py:506, 657-664; tools.py:191-201)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if not k.startswith("GLE_")}
    env.update({k: str(v) for k, v in kw.items()})
    return env


@pytest.mark.parametrize("stream", [False, True])
def test_md_run_two_ranks_gloo_matches_one_rank(tmp_path, stream):
    """stream: the noise through the streamed-factor path, whose factorisations the two ranks split
    (noise.NodeShare: each computes its block once, the node exchanges them in shared memory) --
    the same noise bit for bit, so the same kappa as one rank factorising everything."""
    sys.path.insert(0, HERE)
    from multirank_child import run_md

    kap1, p1, q1 = run_md(str(tmp_path / "one"), 8, 0, stream=stream)
    port = _free_port()
    out = str(tmp_path / "res")
    procs = []
    for r in range(2):
        env = _env(RANK=r, LOCAL_RANK=r, WORLD_SIZE=2, MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "multirank_child.py"), str(tmp_path), out,
                                       "4", "gloo"] + (["stream"] if stream else []), env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    res = []
    for pr in procs:
        o, e = pr.communicate(timeout=240)
        assert pr.returncode == 0, o[-2000:] + e[-3000:]
        res.append(json.loads(o.strip().splitlines()[-1]))
    assert sorted(x["rank"] for x in res) == [0, 1] and all(x["world"] == 2 for x in res)
    r0, r1 = np.load(out + ".rank0.npz"), np.load(out + ".rank1.npz")
    assert kap1.shape == (2, 2) and np.all(np.isfinite(kap1))
    # the reduced per-run kappa is the same on both ranks and equals the one-rank ensemble's
    assert np.array_equal(r0["kap"], r1["kap"])
    assert rel(r0["kap"], kap1) < 1e-12, (r0["kap"], kap1)
    assert rel(np.concatenate([r0["p"], r1["p"]]), p1) < 1e-9
    assert rel(np.concatenate([r0["q"], r1["q"]]), q1) < 1e-9
    if stream:  # each dense factor computed once over both ranks
        n = [int(np.load(str(tmp_path / ("rank%d" % r) / "factorisations.npy"))[0]) for r in range(2)]
        assert min(n) > 0 and abs(n[0] - n[1]) <= 64, n


def test_bench_gpus2_spawns_two_ranks(tmp_path):
    """bench.py --gpus 2 without WORLD_SIZE: the parent starts 2 ranks (torch.distributed.run) and
    the line reports the live group (n_gpus 2, 128 trajectories in all at 64 per rank)."""
    env = _env()
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--same-device",
                        "--dist-backend", "gloo", "--steps", "8", "--warmup", "2", "--fill", "16",
                        "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=400, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["ntraj_total"] == 128, res
    assert res["config"]["parallelism"] == "ensemble-dp2"
    assert res["value"] > 0 and np.isfinite(res["value"])


def _bench_line(r):
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_world1_nccl_under_torchrun(tmp_path):
    """The driver's multi-GPU launch shape on one GPU: `torchrun --nproc-per-node 1 bench.py --gpus 1`
    joins a world-1 nccl (RCCL) process group, so RCCL's communicator and torch's stream pools exist
    beside the stepper's streams, and the window is bracketed by RCCL barriers.  The line must report
    the group and stay at the plain run's rate: the bound (70 us/step at C3, 20 steps) sits between
    the plain line (~50 us) and the hardware-queue sharing trap of profiles/r04 (~115 us)."""
    env = _env(HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "20", "--warmup", "5", "--no-cpu-baseline", "--noise", "white"]
    res = _bench_line(subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400, cwd=str(tmp_path)))
    assert res["n_gpus"] == 1 and res["config"]["ntraj_total"] == 64
    assert res["ensemble_reduce"]["backend"] == "nccl" and res["ensemble_reduce"]["world"] == 1
    assert res["ms_per_step"] < 0.070, res["ms_per_step"]


def test_bench_eight_ranks_same_device_gloo(tmp_path):
    """The 8-GPU ensemble's control flow rehearsed on one GPU: 8 ranks of 8 trajectories on device 0
    over gloo report the live group (n_gpus 8, 64 trajectories in all) and one line."""
    env = _env()
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "2"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--same-device",
                        "--dist-backend", "gloo", "--ntraj", "8", "--noise", "white", "--steps", "8", "--warmup", "2",
                        "--fill", "16", "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=600,
                       cwd=str(tmp_path))
    res = _bench_line(r)
    assert res["n_gpus"] == 8 and res["config"]["ntraj_total"] == 64, res
    assert res["config"]["parallelism"] == "ensemble-dp8"
    assert res["value"] > 0 and np.isfinite(res["value"])
