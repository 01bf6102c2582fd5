#!/bin/bash
# experiment libraries x GLE_* variants, one process per (lib, variant), interleaved over rounds
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/libs.jsonl
for r in $(seq 1 ${ROUNDS:-1}); do
  for lib in ${LIBS:?}; do
    SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_$lib.so timeout -k 10 300 python scripts/exp_time.py --tag $lib --variants "${VARIANTS:-}" >> gpurun_out/libs.jsonl 2>> gpurun_out/libs.err || { echo "lib $lib failed"; tail -20 gpurun_out/libs.err; exit 1; }
  done
done
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/libs.jsonl"):
    d = json.loads(l)
    agg[(d["tag"], d["variant"])].append((d["ms_per_step"] * 1e3, d["short_ms_per_step"] * 1e3))
for v, xs in agg.items():
    print("%-8s %-40s long %s" % (v[0], v[1] or "(default)", " ".join("%.2f" % x[0] for x in xs)))
PY
grep "chain dbg" gpurun_out/libs.err | head -60 || true
