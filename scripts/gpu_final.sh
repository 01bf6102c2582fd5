#!/bin/bash
# round-end evidence: parity suite -> bench (default window, CPU baseline) -> rocprofv3 kernel trace
# + stats of the same bench command -> summaries under gpurun_out/ (copied to profiles/ by hand)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 bench.py --no-cpu-baseline > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err || { echo "prof failed"; tail -20 gpurun_out/prof/bench.err; exit 1; }
N=$(python3 -c "import json;print(json.load(open('gpurun_out/prof/bench.json'))['roofline']['launches'])")
python3 scripts/trace_summary.py gpurun_out/prof/run_kernel_trace.csv --steps --gaps --last cgemm $N > gpurun_out/prof/summary.txt
tail -30 gpurun_out/prof/summary.txt
