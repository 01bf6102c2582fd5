"""Child process of tests/test_gpu_rccl.py: one-rank torch.distributed "nccl" (RCCL) group, then
the same md.Run as the parent's comm-free run; writes the results to an .npz and prints one JSON
line.  argv: work directory, output file."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]


def main():
    import torch
    import torch.distributed as dist

    from test_gpu_rccl import _run_md  # the parent's exact md set-up
    from sclmd_amd import ensemble

    work, out = sys.argv[1], sys.argv[2]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        v = np.array([1.5, -2.0, 3.25])
        ident = bool(np.array_equal(ensemble.allreduce_sums(v, device=0), v))
        import pathlib

        kap, p, q, power, rows, files = _run_md(pathlib.Path(work), None, "nccl")
        info = {"backend": dist.get_backend(), "world": dist.get_world_size(), "allreduce_identity": ident}
    finally:
        dist.destroy_process_group()
    np.savez(out, kap=kap, p=p, q=q, power=power, files=json.dumps(files),
             **{"row%d" % i: r for i, r in enumerate(rows)})
    print(json.dumps(info), flush=True)


if __name__ == "__main__":
    main()
