#!/bin/bash
# round-2 evidence, part 2: C5 bench lines (streamed device noise), PMC HBM traffic of the
# roofline kernel (part 1, scripts/gpu_r02.sh, has the tests, C3/C2 lines and the rocprof trace).  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof gpurun_out/c5
timeout -k 10 300 python -u bench.py --config C5 --ntraj 32 --steps 64 --warmup 8 --no-cpu-baseline > gpurun_out/c5/bench_c5_64.json 2> gpurun_out/c5/bench_c5_64.err || { echo "c5 64 failed"; tail -20 gpurun_out/c5/bench_c5_64.err; exit 1; }
timeout -k 10 300 python -u bench.py --config C5 --ntraj 32 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c5/bench_c5_20.json 2> gpurun_out/c5/bench_c5_20.err || { echo "c5 20 failed"; tail -20 gpurun_out/c5/bench_c5_20.err; exit 1; }
bash scripts/gpu_pmc.sh && cat gpurun_out/pmc/traffic.json
