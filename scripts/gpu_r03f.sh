#!/bin/bash
# interference mechanism: cgemm holding its slots without MFMAs (sleep, CG_DBG=15) vs pure-MFMA
# cgemm (7) vs none (SKIP=1); chain with 4 accumulator sets (CH_NA=4) beside the ladder
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 400 python scripts/exp_time.py --steps 512 --rounds 2 --variants "GLE_CG_PER_CU=0.5;GLE_CG_DBG=15;GLE_CG_DBG=7;GLE_DBG_SKIP=1" > gpurun_out/r03/mech.jsonl 2> gpurun_out/r03/mech.err || { echo "mech failed"; tail -20 gpurun_out/r03/mech.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r03/mech.jsonl'):
    d=json.loads(l); print('%-22s'%d['variant'], d['round'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'])
"
for lib in na4 exp na4 exp; do
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_$lib.so timeout -k 10 200 python scripts/exp_time.py --steps 512 --tag $lib > gpurun_out/r03/n_$lib.json 2>/dev/null || { echo "lib $lib failed"; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/r03/n_$lib.json').read()); print('$lib', 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'])
"
done
