#!/bin/bash
# interference anatomy (background schedule): which part of the far field slows the chain
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
export SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so
timeout -k 10 500 python scripts/exp_time.py --steps 512 --rounds 2 --variants "GLE_CG_PER_CU=0.5;GLE_CG_DBG=1;GLE_CG_DBG=4;GLE_CG_DBG=7;GLE_DBG_SKIP=1;GLE_DBG_SKIP=6;GLE_DBG_NO_LADDER=1;GLE_CG_PER_CU=2" > gpurun_out/r03/interf.jsonl 2> gpurun_out/r03/interf.err || { echo "interf failed"; tail -20 gpurun_out/r03/interf.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r03/interf.jsonl'):
    d=json.loads(l); print('%-22s'%d['variant'], d['round'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'])
"
for lib in wpe5 exp wpe5 exp; do
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_$lib.so timeout -k 10 200 python scripts/exp_time.py --steps 512 --tag $lib > gpurun_out/r03/lib_$lib.json 2>/dev/null || { echo "lib $lib failed"; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/r03/lib_$lib.json').read()); print('$lib', 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'])
"
done
