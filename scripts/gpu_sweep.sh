#!/bin/bash
# plan-knob sweep (experiment build, GLE_* / EXP_* variants interleaved over rounds in one process)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
V=${VARIANTS:?}
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 900 python scripts/exp_time.py --variants "$V" --rounds ${ROUNDS:-2} --tag sweep > gpurun_out/sweep.jsonl 2> gpurun_out/sweep.err || { echo "sweep failed"; tail -20 gpurun_out/sweep.err; exit 1; }
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/sweep.jsonl"):
    d = json.loads(l)
    agg[d["variant"]].append((d["ms_per_step"] * 1e3, d["short_ms_per_step"] * 1e3, d["finite"]))
for v, xs in agg.items():
    print("%-40s long %s short %s" % (v or "(default)", " ".join("%.2f" % x[0] for x in xs), " ".join("%.2f" % x[1] for x in xs)), all(x[2] for x in xs))
PY
