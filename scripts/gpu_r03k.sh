#!/bin/bash
# fewer background launches: one GEMM launch per level block (grid-stride over its items, grid cap)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 700 python scripts/exp_time.py --chainprof 1 --steps 512 --rounds 2 --short-reps 3 --variants "GLE_CG_PER_CU=0.5;GLE_NO_PIECES=1,GLE_BG_GRID=128;GLE_NO_PIECES=1,GLE_BG_GRID=256;GLE_NO_PIECES=1,GLE_BG_GRID=64;GLE_NO_PIECES=1;GLE_PIECE_STEP=8" > gpurun_out/r03/fewl.jsonl 2> gpurun_out/r03/fewl.err || { echo "failed"; tail -20 gpurun_out/r03/fewl.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r03/fewl.jsonl'):
    d=json.loads(l); print('%-40s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'chain us/step %.1f'%d.get('chain_us_per_step',0), d['short_reps_ms'], d['finite'])
"
