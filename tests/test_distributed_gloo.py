"""N > 1 ensemble path on CPU: 2 gloo ranks each step their shard of the trajectory ensemble (the
oracle stands in for the device here) and combine the per-run heat-current statistics with the
product's single all-reduce; the result equals the unsharded ensemble."""
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def ensemble_sums(offset, count):
    """Per-bath [sum_b mean_t cur, sum_b mean^2, count] for trajectories offset..offset+count."""
    from conftest import load_golden, oracle_from_golden

    g = load_golden("vv_twoph")
    nmd = int(g["nmd"])
    out = np.zeros((int(g["nbath"]), 3))
    for b in range(offset, offset + count):
        sim = oracle_from_golden(g)
        rng = np.random.default_rng(100 + b)
        sim.p = sim.p * (1 + 0.1 * rng.normal())
        for bath in sim.baths:
            bath.noise = bath.noise * (1 + rng.normal())
        for _ in range(nmd):
            sim.step()
        for i, bath in enumerate(sim.baths):
            m = np.mean(bath.cur)
            out[i] += [m, m * m, 1.0]
    return out


def _worker(rank, world, port, ntot, q):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    import torch.distributed as dist

    from sclmd_amd import ensemble

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    off, cnt = ensemble.shard(ntot, rank, world)
    red = ensemble.allreduce_sums(ensemble_sums(off, cnt))
    q.put((rank, red))
    dist.destroy_process_group()


def test_two_rank_ensemble_reduce():
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ntot = 5
    ps = [ctx.Process(target=_worker, args=(r, 2, port, ntot, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = ensemble_sums(0, ntot)
    for r in range(2):
        np.testing.assert_allclose(res[r], full, rtol=1e-12, atol=0)
    from sclmd_amd.ensemble import ensemble_stats

    mean, err = ensemble_stats(full)
    assert mean.shape == (2,) and np.all(err >= 0)
