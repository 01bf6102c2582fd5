#!/bin/bash
# parity tests -> bench -> rocprofv3 kernel trace; stops at the first failure
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/peak_probe > gpurun_out/peak.json 2>&1; cat gpurun_out/peak.json
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 900 python bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
mkdir -p gpurun_out/prof
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 bench.py --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err || { echo "prof failed"; tail -20 gpurun_out/prof/bench.err; exit 1; }
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/prof/run_kernel_stats.csv')))
for r in rows:
    print("%-60s %6s %10.1f %9.1f %5.1f%%"%(r['Name'][:60], r['Calls'], float(r['TotalDurationNs'])/1e3, float(r['AverageNs'])/1e3, float(r['Percentage'])))
PY
