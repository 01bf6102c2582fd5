#!/bin/bash
# GLE ensemble current vs Landauer over a few settings, then the GPU test
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/landauer_check.py > gpurun_out/landauer.jsonl 2> gpurun_out/landauer.err || { tail -5 gpurun_out/landauer.err; exit 1; }
cat gpurun_out/landauer.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_negf.py -x -q -m gpu --timeout 200 --timeout-method thread 2>&1 | tail -3
