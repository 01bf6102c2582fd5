#!/usr/bin/env python3
"""MFMA-pipe utilisation per kernel class from one rocprofv3 --pmc pass of SQ_VALU_MFMA_BUSY_CYCLES
and GRBM_GUI_ACTIVE over a bench run (the timed region's last N dispatches of each class).

  utilisation = MFMA busy cycles / (kernel cycles x SIMDs),  kernel cycles = GRBM_GUI_ACTIVE / 8
  (rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs, MI355X_MICROARCH.md DVFS note); 1024 SIMDs.

    python scripts/mfma_summary.py gpurun_out/mfma/run_counter_collection.csv N OUT.json
"""
import collections
import csv
import json
import sys

SIMDS = 256 * 4


def main():
    path, last, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    per = collections.defaultdict(dict)   # dispatch -> {counter: value, "kernel": name}
    for r in csv.DictReader(open(path)):
        d = int(r.get("Dispatch_Id", r.get("Correlation_Id", 0)))
        per[d]["kernel"] = r["Kernel_Name"]
        per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    classes = {"cgemm_kernel": "cgemm", "chain_kernel": "chain", "contract_kernel": "contract",
               "seg_fft_kernel": "seg_fft", "far_ifft_kernel": "far_ifft"}
    groups = collections.defaultdict(list)
    for d in sorted(per):
        name = per[d]["kernel"]
        for key, cls in classes.items():
            if name.startswith(key) or ("::" + key) in name or (" " + key) in name or key in name.split("<")[0]:
                groups[cls].append(per[d])
                break
    res = {"method": __doc__.strip().splitlines()[0], "simds": SIMDS, "classes": {}}
    for cls, rows in groups.items():
        rows = rows[-last:] if cls == "cgemm" else rows[-(last * 4):]
        busy = sum(r.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for r in rows)
        cyc = sum(r.get("GRBM_GUI_ACTIVE", 0.0) for r in rows) / 8.0
        res["classes"][cls] = {"dispatches": len(rows), "mfma_busy_cycles": busy,
                               "kernel_cycles": cyc, "mfma_util": busy / max(cyc * SIMDS, 1.0)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
