"""bench.py's multi-GPU launch contract (no GPU needed): --gpus N > 1 without a torchrun environment
starts N ranks through torch.distributed.run on the loopback rendezvous, a rank whose WORLD_SIZE
differs from --gpus refuses before any GPU call, and the experiment environment is refused."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _run(args, env_extra):
    env = {k: v for k, v in os.environ.items() if not k.startswith("GLE_") and k not in ("WORLD_SIZE", "RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=120)


def test_world_size_mismatch_refused():
    r = _run(["--gpus", "2", "--steps", "1"], {"WORLD_SIZE": "4", "RANK": "0"})
    assert r.returncode != 0
    assert "--gpus 2 but WORLD_SIZE=4" in r.stderr


def test_experiment_env_refused():
    r = _run(["--steps", "1"], {"GLE_PLAN_VARIANT": "1"})
    assert r.returncode != 0 and "refusing" in r.stderr


def test_spawn_command_shape():
    import bench

    cmd = bench.spawn_command(4, ["--gpus", "4", "--steps", "20"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    assert cmd[-5].endswith("bench.py") and cmd[-4:] == ["--gpus", "4", "--steps", "20"]


def test_rank_env_matching_gpus_is_a_rank(monkeypatch):
    import argparse

    import bench

    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.launch_or_check_world(argparse.Namespace(gpus=2), []) is None
    monkeypatch.delenv("WORLD_SIZE")
    assert bench.launch_or_check_world(argparse.Namespace(gpus=1), []) is None
