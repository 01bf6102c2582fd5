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


def _plan_arrays(segs):
    """A streamed factor plan as comparable (kind, w0, arrays...) tuples."""
    out = []
    for seg in segs:
        if seg[0] == "shared":
            out.append(("shared", seg[1], seg[2], np.array(seg[3]), np.array(seg[4])))
        else:
            m = seg[2]
            out.append(("dense", seg[1]) + (tuple(np.array(x) for x in m) if isinstance(m, tuple) else (np.array(m),)))
    return out


def _share_baths():
    from sclmd_amd import synthetic

    rng = np.random.default_rng(21)
    nmd = 256
    return [synthetic.make_phbath(300.0, list(range(12)), 6, nmd, rng, nw=30),
            synthetic.make_biased_ebath(300.0, list(range(10)), nmd, rng)]


def _share_worker(rank, world, port, root, q):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    import torch.distributed as dist

    from sclmd_amd import noise as Nz

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res, counts = [], []
    for b, chunk in [(b, c) for c in (16, 2) for b in _share_baths()]:  # chunk 2: runs inside one block
        sh = Nz.NodeShare(rank, world, dist.barrier, "t%d" % port, root=root)
        cache = {}
        res.append(_plan_arrays(Nz.stream_factor_plan(b, chunk=chunk, workers=2, cache=cache, share=sh)))
        counts.append(sh.computed)
        assert cache["complete"] and len(cache["segments"]) == len(res[-1])
    q.put((rank, res, counts))
    dist.destroy_process_group()


def test_node_share_splits_factorisation_and_matches_one_rank(tmp_path):
    """Three ranks factorise a phonon and a biased electron bath's noise spectra together
    (noise.NodeShare): each computes its block of the dense frequencies once, the blocks
    go through node-local files, and every rank's plan is bitwise the one-rank plan; the files are
    gone afterwards."""
    import multiprocessing as mp

    from sclmd_amd import noise as Nz

    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_share_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict((r, (res, cnt)) for r, res, cnt in (q.get(timeout=300) for _ in range(world)))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert os.listdir(tmp_path) == []
    for k, (b, chunk) in enumerate([(b, c) for c in (16, 2) for b in _share_baths()]):
        want = _plan_arrays(Nz.stream_factor_plan(b, chunk=chunk, workers=2))
        ndense = sum(s[2].shape[0] for s in want if s[0] == "dense")
        assert sum(got[r][1][k] for r in range(world)) == ndense  # each factor computed once on the node
        assert max(got[r][1][k] for r in range(world)) <= ndense // world + 1
        for r in range(world):
            plan = got[r][0][k]
            assert len(plan) == len(want)
            for a, w in zip(plan, want):
                assert a[0] == w[0] and a[1] == w[1]
                for x, y in zip(a[2:], w[2:]):
                    assert np.array_equal(np.asarray(x), np.asarray(y))


def _fac_bath():
    from sclmd_amd import synthetic

    return synthetic.make_phbath(300.0, list(range(64)), 6, 2048, np.random.default_rng(5), nw=30)


def _fac_worker(rank, world, port, root, q):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    import torch.distributed as dist

    from sclmd_amd import noise as Nz

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = Nz.NodeShare(rank, world, dist.barrier, "f%d" % port, root=root)
    f = _fac_bath().noise_factor(share=sh)
    q.put((rank, f.evals, f.evecs, sh.computed))
    dist.destroy_process_group()


def test_node_share_resident_factor_matches_one_rank(tmp_path):
    """The resident path's eigendecomposition of every nonzero frequency (bath.noise_factor, e.g. C3's
    phonon baths) split over 3 ranks by frequency blocks: each rank's factor is bitwise the one-rank
    one."""
    import multiprocessing as mp

    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_fac_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for p in ps:
        p.start()
    got = [q.get(timeout=300) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert os.listdir(tmp_path) == []
    b = _fac_bath()
    want = b.noise_factor()
    spec = b._spectrum()
    nonzero = int(np.count_nonzero(spec.reshape(spec.shape[0], -1).any(axis=1)))
    assert sum(g[3] for g in got) == nonzero  # each nonzero frequency decomposed once on the node
    for _, ev, vec, _ in got:
        assert np.array_equal(ev, want.evals) and np.array_equal(vec, want.evecs)
