#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run -> gpurun_out/prof/
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 bench.py --no-cpu-baseline "$@" > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err
