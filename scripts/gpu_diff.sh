#!/bin/bash
# bench vs exp_time on one box: noise content (device coloured vs white) and harness differences
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/diff
timeout -k 10 300 python bench.py --no-cpu-baseline --noise white > gpurun_out/diff/white.json 2> gpurun_out/diff/white.err || { echo "white failed"; tail -20 gpurun_out/diff/white.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/diff/dev.json 2> gpurun_out/diff/dev.err || { echo "dev failed"; tail -20 gpurun_out/diff/dev.err; exit 1; }
timeout -k 10 300 python scripts/exp_time.py --rounds 2 > gpurun_out/diff/exp.jsonl 2> gpurun_out/diff/exp.err || { echo "exp failed"; tail -20 gpurun_out/diff/exp.err; exit 1; }
python3 - <<'PY'
import json
for f in ["white", "dev"]:
    d = json.load(open("gpurun_out/diff/%s.json" % f))
    print(f, "%.2f us/step" % (d["ms_per_step"] * 1e3), "roof %.3f" % d["roofline"]["frac"])
for l in open("gpurun_out/diff/exp.jsonl"):
    d = json.loads(l); print("exp", "%.2f us/step" % (d["ms_per_step"] * 1e3))
PY
