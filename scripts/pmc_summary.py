#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per launch of the
dominant kernel.  gfx950 correction (MI355X_MICROARCH.md, HBM section; re-calibrated here with
tools/peak_probe's known 4 GiB read streams: 8 B/lane and 16 B/lane coalesced reads both report
exactly half): hbm_read = 2 * FETCH_SIZE * 1024, hbm_write = WRITE_SIZE * 1024.

    python scripts/pmc_summary.py gpurun_out/pmc OUT.json --kernel 'contract_kernel<16' \
        --config C3 --ntraj 64
"""
import argparse
import csv
import json
import os


def per_launch(path, kernel, last=0, skip=0):
    """Counter value per dispatch of `kernel`, in dispatch order; last > 0 keeps only `last`
    dispatches before the newest `skip` (bench.py's roofline window is followed by one more window
    of the same steps, the chain stamps: skip = last)."""
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id", r.get("Correlation_Id", 0))))
    vals = [float(r["Counter_Value"]) for r in rows]
    if last <= 0:
        return vals
    return vals[len(vals) - last - skip:len(vals) - skip]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmcdir")
    ap.add_argument("out")
    ap.add_argument("--kernel", default="cgemm_kernel")
    ap.add_argument("--config", default="C3")
    ap.add_argument("--ntraj", type=int, default=64)
    ap.add_argument("--far-mode", default="spectral")
    ap.add_argument("--skip-chain-window", type=int, default=1,
                    help="1: the newest `last` dispatches are bench.py's chain-stamp window; skip them")
    ap.add_argument("--last", type=int, default=-1,
                    help="dispatches of the timed region (default: the bench JSON's roofline.launches)")
    a = ap.parse_args()
    last = a.last
    if last < 0:
        try:
            last = int(json.load(open(os.path.join(a.pmcdir, "FETCH_SIZE.json")))["roofline"]["launches"])
        except (OSError, ValueError, KeyError):
            last = 0
    skip = last if a.skip_chain_window else 0
    f = per_launch(os.path.join(a.pmcdir, "FETCH_SIZE", "run_counter_collection.csv"), a.kernel, last, skip)
    w = per_launch(os.path.join(a.pmcdir, "WRITE_SIZE", "run_counter_collection.csv"), a.kernel, last, skip)
    fetch = sum(f) / len(f) * 1024.0
    write = sum(w) / len(w) * 1024.0
    res = {"config": a.config, "ntraj": a.ntraj, "far_mode": a.far_mode, "kernel": a.kernel,
           "launches": [len(f), len(w)],
           "fetch_size_bytes_raw": fetch, "write_size_bytes": write,
           "hbm_bytes_per_launch": 2.0 * fetch + write,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                     "read bytes = 2 x FETCH_SIZE (gfx950 half-count, calibrated on 4 GiB 8 B/lane and "
                     "16 B/lane streams), write bytes = WRITE_SIZE"}
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
