#!/bin/bash
# experiment libraries (compile-time variants) interleaved over rounds, one process per measurement
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/libs.jsonl
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in ${LIBS:?}; do
    SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_$lib.so timeout -k 10 120 python scripts/exp_time.py --tag $lib >> gpurun_out/libs.jsonl 2>> gpurun_out/libs.err || { echo "lib $lib failed"; tail -20 gpurun_out/libs.err; exit 1; }
  done
done
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/libs.jsonl"):
    d = json.loads(l)
    agg[d["tag"]].append((d["ms_per_step"] * 1e3, d["short_ms_per_step"] * 1e3, d["finite"]))
for v, xs in agg.items():
    print("%-12s long %s short %s" % (v, " ".join("%.2f" % x[0] for x in xs), " ".join("%.2f" % x[1] for x in xs)), all(x[2] for x in xs))
PY
