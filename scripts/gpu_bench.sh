#!/bin/bash
# 1-GPU bench on the box (bounded), JSON line -> gpurun_out/bench.json
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
