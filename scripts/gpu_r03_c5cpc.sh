#!/bin/bash
# C5 far-field GEMM chunk sizes (workgroups per CU per chunk), one process, interleaved rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03c5cpc
mkdir -p $O
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 1000 python -u scripts/exp_time.py --config C5 --ntraj 32 --steps 256 --rounds 2 --variants "GLE_CG_PER_CU=4;GLE_CG_PER_CU=8;GLE_CG_PER_CU=16;GLE_CG_PER_CU=32" --tag c5cpc > $O/c5cpc.jsonl 2> $O/c5cpc.err || { echo "c5cpc failed"; tail -20 $O/c5cpc.err; exit 1; }
python3 -c "
import json
for l in open('$O/c5cpc.jsonl'):
    d=json.loads(l); print('%-20s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], d['finite'])
"
