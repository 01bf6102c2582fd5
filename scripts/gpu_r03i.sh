#!/bin/bash
# is it the far-field launches themselves? cgemm chunks replaced by empty one-workgroup launches
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 600 python scripts/exp_time.py --chainprof 1 --steps 512 --rounds 2 --variants "GLE_CG_PER_CU=0.5;GLE_CG_DBG=15;GLE_CG_DBG=16;GLE_DBG_SKIP=1;GLE_DBG_SKIP=7;GLE_DBG_NO_LADDER=1" > gpurun_out/r03/launchx.jsonl 2> gpurun_out/r03/launchx.err || { echo "failed"; tail -20 gpurun_out/r03/launchx.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r03/launchx.jsonl'):
    d=json.loads(l); print('%-30s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'chain us/step %.1f'%d.get('chain_us_per_step',0))
"
