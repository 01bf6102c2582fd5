#!/usr/bin/env python3
"""Per-rank host factorisation time of the streamed C5 noise spectra when the ranks of one node split
them (noise.NodeShare), without a GPU.  For each bath of the C5 junction: the one-rank
time (every dense factor on this process's thread pool) and, for a node of --world ranks, each rank's
block of the dense frequencies timed alone on the same pool (a rank of the 8-GPU node has its own
cores: the node's ranks run their blocks at once).  Factors are the same calls either way
(tests/test_distributed_gloo.py checks the bitwise equality); the exchange through shared memory is
timed as a write plus a read of the whole factor set.

    python scripts/noise_share_timing.py --world 8 [--workers 16]

Prints one JSON line."""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--config", default="C5")
    args = ap.parse_args()
    from sclmd_amd import noise as Nz
    from sclmd_amd import synthetic

    _, _, baths, meta = synthetic.junction(args.config, seed=1234, gmem_device=True)
    out = {"config": args.config, "world": args.world, "workers_per_rank": args.workers,
           "cpu": os.uname().machine, "baths": []}
    tot1, totr = 0.0, [0.0] * args.world
    for b in baths:
        nfreq = int(b.nmd / 2) + 1
        dtype = complex if b.kind == "ebath" else float
        dense = [i for i in range(nfreq) if b._spectrum_term(i, matrix=False)[0] == "dense"]
        t0 = time.perf_counter()
        facs = Nz._dense_factors(b, dense, dtype, args.workers)
        t1 = time.perf_counter() - t0
        blocks = []
        sh = Nz.NodeShare(0, args.world, lambda: None, "timing")
        for r in range(args.world):
            lo, hi = sh.block(len(dense), r)
            t0 = time.perf_counter()
            Nz._dense_factors(b, dense[lo:hi], dtype, args.workers)
            blocks.append(time.perf_counter() - t0)
        # the exchange: every block written once and read by every rank (one read timed here)
        arr = np.stack(facs)
        del facs
        with tempfile.TemporaryDirectory(dir=sh.root) as d:
            f = os.path.join(d, "fac.npy")
            t0 = time.perf_counter()
            np.save(f, arr)
            tw = time.perf_counter() - t0
            t0 = time.perf_counter()
            np.array(np.load(f, mmap_mode="r"))
            tr = time.perf_counter() - t0
        nbytes = arr.nbytes
        del arr
        out["baths"].append({"kind": b.kind, "nc": b.nc, "nfreq": nfreq, "dense": len(dense),
                             "one_rank_s": round(t1, 3), "rank_block_s": [round(x, 3) for x in blocks],
                             "exchange_bytes": nbytes, "write_s": round(tw, 3), "read_s": round(tr, 3)})
        tot1 += t1
        for r in range(args.world):
            totr[r] += blocks[r] + tr + tw / args.world
    out["one_rank_total_s"] = round(tot1, 3)
    out["per_rank_total_s"] = [round(x, 3) for x in totr]
    out["per_rank_max_s"] = round(max(totr), 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
