#!/bin/bash
# GPU parity suite, then the experiment list and a kernel trace with the gap analysis
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash scripts/gpu_exp_prof.sh "$@"
