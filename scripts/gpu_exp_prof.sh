#!/bin/bash
# experiment list (scripts/gpu_exp.sh) and a kernel trace of the default build with the gap analysis
set -o pipefail
export TMPDIR=/tmp
bash scripts/gpu_exp.sh "$@" || exit 1
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof -o run -- \
  python3 bench.py --no-cpu-baseline --steps 200 --warmup 20 > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err || { echo "prof failed"; tail -20 gpurun_out/prof/bench.err; exit 1; }
python3 scripts/trace_summary.py gpurun_out/prof/run_kernel_trace.csv --steps --gaps > gpurun_out/prof/summary.txt
tail -28 gpurun_out/prof/summary.txt
