#!/bin/bash
# near-field side stream experiment: GLE_NEAR_SIDE off/on at several hardware-queue counts
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/side.jsonl
for q in 4 5 8; do
  GPU_MAX_HW_QUEUES=$q SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 300 python scripts/exp_time.py --tag "q$q" --variants ";GLE_NEAR_SIDE=1" --rounds 2 >> gpurun_out/side.jsonl 2>> gpurun_out/side.err || { echo "side q$q failed"; tail -20 gpurun_out/side.err; exit 1; }
done
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/side.jsonl"):
    d = json.loads(l)
    agg[(d["tag"], d["variant"])].append((d["ms_per_step"] * 1e3, d["short_ms_per_step"] * 1e3, d["finite"]))
for v, xs in agg.items():
    print("%-4s %-20s long %s short %s" % (v[0], v[1] or "(default)", " ".join("%.2f" % x[0] for x in xs), " ".join("%.2f" % x[1] for x in xs)), all(x[2] for x in xs))
PY
