#!/bin/bash
# parity tests -> rocprofv3 kernel trace of a short bench (per-launch breakdown via trace_summary.py)
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 bench.py --no-cpu-baseline --steps 128 --warmup 16 "$@" > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err || { echo "prof failed"; tail -20 gpurun_out/prof/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/prof/bench.json'));print('value',d['value'],'ms/step',d['ms_per_step'])"
python3 scripts/trace_summary.py gpurun_out/prof/run_kernel_trace.csv
