#!/bin/bash
# GPU parity suite on the box (one process, bounded).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu "$@" > gpurun_out/gpu_tests.log 2>&1
