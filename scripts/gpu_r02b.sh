#!/bin/bash
# round-2 evidence, part 2: C5 bench lines (streamed device noise), rocprofv3 kernel trace + stats
# of the default bench, PMC HBM traffic of the roofline kernel.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof gpurun_out/c5
timeout -k 10 300 python -u bench.py --config C5 --ntraj 32 --steps 64 --warmup 8 --no-cpu-baseline > gpurun_out/c5/bench_c5_64.json 2> gpurun_out/c5/bench_c5_64.err || { echo "c5 64 failed"; tail -20 gpurun_out/c5/bench_c5_64.err; exit 1; }
timeout -k 10 300 python -u bench.py --config C5 --ntraj 32 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c5/bench_c5_20.json 2> gpurun_out/c5/bench_c5_20.err || { echo "c5 20 failed"; tail -20 gpurun_out/c5/bench_c5_20.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 bench.py --no-cpu-baseline > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err || { echo "prof failed"; tail -20 gpurun_out/prof/bench.err; exit 1; }
N=$(python3 -c "import json;print(json.load(open('gpurun_out/prof/bench.json'))['roofline']['launches'])")
python3 scripts/trace_summary.py gpurun_out/prof/run_kernel_trace.csv --steps --gaps --last cgemm $N > gpurun_out/prof/summary.txt
tail -12 gpurun_out/prof/summary.txt
bash scripts/gpu_pmc.sh && cat gpurun_out/pmc/traffic.json
