#!/bin/bash
# GPU parity suite, then the bench (short CPU baseline) and the steady-state trace summary
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --cpu-budget 5 "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 bench.py --no-cpu-baseline --steps 200 --warmup 20 > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err || { echo "prof failed"; tail -20 gpurun_out/prof/bench.err; exit 1; }
python3 scripts/trace_summary.py gpurun_out/prof/run_kernel_trace.csv --steps --last cgemm $(python3 -c "import json;print(json.load(open('gpurun_out/prof/bench.json'))['roofline']['launches'])") > gpurun_out/prof/summary.txt
tail -22 gpurun_out/prof/summary.txt
