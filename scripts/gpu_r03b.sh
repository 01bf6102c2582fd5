#!/bin/bash
# round-3 diagnostics: f64 MFMA issue/dependency probe; the two suite-order failures fixed; chain
# timelines (per-tile stamps) at C3 alone and beside the ladder (experiment build).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 60 ./tools/mfma_probe > gpurun_out/r03/mfma_probe.jsonl 2>&1 || { echo "probe failed"; cat gpurun_out/r03/mfma_probe.jsonl; exit 1; }
cat gpurun_out/r03/mfma_probe.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_noise_stream.py tests/test_gpu_rccl.py -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r03/fix_tests.log 2>&1 || { echo "fix tests failed"; tail -40 gpurun_out/r03/fix_tests.log; exit 1; }
tail -2 gpurun_out/r03/fix_tests.log
export SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so
GLE_DBG_NO_LADDER=1 GLE_CHAIN_DBG=600 timeout -k 10 300 python scripts/exp_time.py --steps 512 > gpurun_out/r03/chain_alone.json 2> gpurun_out/r03/chain_alone.err || { echo "alone failed"; tail -20 gpurun_out/r03/chain_alone.err; exit 1; }
cat gpurun_out/r03/chain_alone.json; grep "chain dbg" gpurun_out/r03/chain_alone.err
GLE_CHAIN_DBG=600 timeout -k 10 300 python scripts/exp_time.py --steps 512 > gpurun_out/r03/chain_ladder.json 2> gpurun_out/r03/chain_ladder.err || { echo "ladder failed"; tail -20 gpurun_out/r03/chain_ladder.err; exit 1; }
cat gpurun_out/r03/chain_ladder.json; grep "chain dbg" gpurun_out/r03/chain_ladder.err
GLE_CHAIN_DBG=601 timeout -k 10 300 python scripts/exp_time.py --steps 512 > gpurun_out/r03/chain_ladder2.json 2> gpurun_out/r03/chain_ladder2.err || { echo "ladder2 failed"; exit 1; }
grep "chain dbg" gpurun_out/r03/chain_ladder2.err
