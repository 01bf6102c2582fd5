#!/bin/bash
# chain kernel time per step vs step time in the interference variants; k-split background items
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 700 python scripts/exp_time.py --chainprof 1 --steps 512 --rounds 1 --short-reps 3 --variants "GLE_CG_PER_CU=0.5;GLE_CG_DBG=15;GLE_DBG_SKIP=1;GLE_DBG_NO_LADDER=1;GLE_CU_SPLIT=64;GLE_CU_SPLIT=64,GLE_DBG_NO_LADDER=1;GLE_CU_SPLIT=128,GLE_DBG_NO_LADDER=1;GLE_DBG_SKIP=6;GLE_BG_SPLIT=1;GLE_BG_SPLIT=1,GLE_CG_PER_CU=2;GLE_BG_SPLIT=1,GLE_CG_PER_CU=1;GLE_BG_SPLIT=1,GLE_FAR_KS=16,GLE_CG_PER_CU=2" > gpurun_out/r03/chainprof.jsonl 2> gpurun_out/r03/chainprof.err || { echo "failed"; tail -20 gpurun_out/r03/chainprof.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r03/chainprof.jsonl'):
    d=json.loads(l); print('%-50s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'chain us/step %.1f'%d.get('chain_us_per_step',0), d['short_reps_ms'], d['finite'])
"
