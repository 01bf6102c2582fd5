#!/bin/bash
# disjoint CU sets for the per-step chain (main stream) and the far field (background streams)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 600 python scripts/exp_time.py --steps 512 --rounds 1 --variants "GLE_CG_PER_CU=0.5;GLE_CU_SPLIT=64,GLE_CG_PER_CU=1;GLE_CU_SPLIT=64,GLE_CG_PER_CU=0.5;GLE_CU_SPLIT=96,GLE_CG_PER_CU=1;GLE_CU_SPLIT=96,GLE_CG_PER_CU=1.5;GLE_CU_SPLIT=128,GLE_CG_PER_CU=1;GLE_CU_SPLIT=128,GLE_CG_PER_CU=2;GLE_CU_SPLIT=64,GLE_CU_SPLIT_MAIN=0,GLE_CG_PER_CU=1;GLE_CG_PER_CU=0.5" > gpurun_out/r03/split.jsonl 2> gpurun_out/r03/split.err || { echo "split failed"; tail -20 gpurun_out/r03/split.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r03/split.jsonl'):
    d=json.loads(l); print('%-50s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], d['finite'])
"
bash scripts/gpu_r03f.sh
