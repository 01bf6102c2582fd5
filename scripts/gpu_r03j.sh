#!/bin/bash
# fused far-field schedule with deeper K-hat prefetch and slot-sized launch shares vs background
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 700 python scripts/exp_time.py --chainprof 1 --steps 512 --rounds 2 --variants "GLE_CG_PER_CU=0.5;GLE_FAR_FUSED=1;GLE_FAR_FUSED=1,GLE_FAR_KS=24;GLE_FAR_FUSED=1,GLE_FAR_KS=64;GLE_FAR_FUSED=1,GLE_FAR_AFRAC=0.25" > gpurun_out/r03/fused2.jsonl 2> gpurun_out/r03/fused2.err || { echo "failed"; tail -20 gpurun_out/r03/fused2.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r03/fused2.jsonl'):
    d=json.loads(l); print('%-40s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'chain us/step %.1f'%d.get('chain_us_per_step',0), d['finite'])
"
