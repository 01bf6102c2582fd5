"""Rank process of tests/test_gpu_multirank.py: a torch.distributed group (backend from argv, every rank
on device 0) and md.Run through the HIP stepper on this rank's shard of the ensemble (traj_offset =
rank * ntraj).  Writes this rank's kappa per run, p and q to <out>.rank<r>.npz and prints one JSON
line.  argv: work directory, output prefix, ntraj per rank, backend [, "stream"]."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]


def run_md(workdir, ntraj, traj_offset, comm=None, stream=False):
    """The shared md set-up: small C3-shaped junction, device noise, two runs (md.py:493-682).
    stream: the noise through the streamed-factor path (the C5 path: with several ranks the node's
    ranks split its factorisations, noise.NodeShare)."""
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic

    os.makedirs(workdir, exist_ok=True)
    cwd = os.getcwd()
    os.chdir(workdir)
    try:
        dyn, axyz, baths, meta = synthetic.junction("C3", seed=5, natom=12, ml=64, nmd=128, nw=80)
        m = MD.md(meta["dt"], meta["nmd"], meta["T"], axyz=axyz, dyn=dyn, ntraj=ntraj, seed=41, nstart=0,
                  nstop=2, traj_offset=traj_offset, device=0, noise_mode="device", comm=comm, verbose=False)
        for b in baths:
            m.AddBath(b)
        if stream:
            m.noise_stream_bytes = 0
        m.Run()
        share = getattr(m, "_share", None)
        if share is not None:
            np.save(os.path.join(workdir, "factorisations.npy"), np.array([share.total]))
        kap = np.array(m.kappa_runs)
        p, q = np.array(m.p).reshape(ntraj, -1), np.array(m.q).reshape(ntraj, -1)
        m.close()
    finally:
        os.chdir(cwd)
    return kap, p, q


def main():
    import torch.distributed as dist

    work, out, ntraj, backend = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    stream = len(sys.argv) > 5 and sys.argv[5] == "stream"
    dist.init_process_group(backend)
    r, w = dist.get_rank(), dist.get_world_size()
    try:
        kap, p, q = run_md(os.path.join(work, "rank%d" % r), ntraj, r * ntraj, stream=stream)
        dist.barrier()
    finally:
        dist.destroy_process_group()
    np.savez("%s.rank%d.npz" % (out, r), kap=kap, p=p, q=q)
    print(json.dumps({"rank": r, "world": w, "backend": backend}), flush=True)


if __name__ == "__main__":
    main()
