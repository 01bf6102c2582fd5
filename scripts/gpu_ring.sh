#!/bin/bash
# cgemm prefetch-ring variants (experiment build, GLE_CG_RING=AD*10+XD): step time interleaved over
# rounds, then the cgemm rate from HIP events / device timestamps.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
V=${VARIANTS:-"GLE_CG_RING=0;GLE_CG_RING=31;GLE_CG_RING=32;GLE_CG_RING=51;GLE_CG_RING=52;GLE_CG_RING=72"}
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 600 python scripts/exp_time.py --variants "$V" --rounds ${ROUNDS:-2} --tag ring > gpurun_out/ring.jsonl 2> gpurun_out/ring.err || { echo "ring failed"; tail -20 gpurun_out/ring.err; exit 1; }
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 600 python scripts/exp_time.py --variants "$V" --rounds 1 --profile 1 --tag ringprof > gpurun_out/ringprof.jsonl 2> gpurun_out/ringprof.err || { echo "ringprof failed"; tail -20 gpurun_out/ringprof.err; exit 1; }
python3 - <<'PY'
import json
for f in ["ring", "ringprof"]:
    for l in open("gpurun_out/%s.jsonl" % f):
        d = json.loads(l)
        print(f, d["variant"], d["round"], "%.2f us/step" % (d["ms_per_step"] * 1e3), "short %.2f" % (d["short_ms_per_step"] * 1e3),
              "cgemm %.1f us %.1f TF" % (d.get("cgemm_avg_us", 0), d.get("cgemm_tflops", 0)), d["finite"])
PY
