#!/bin/bash
# C5 (32 trajectories) plan variants, one process, interleaved: 32-column DOF tiles (each matrix
# fragment fetched once instead of once per 16-column tile), 4-wave fused tiles, far-field chunks.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03c5exp
mkdir -p $O
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 900 python -u scripts/exp_time.py --config C5 --ntraj 32 --steps 128 --short 20 --rounds 2 --variants ";GLE_CHAIN_DRN=2;GLE_CHAIN_NW=4,4,4;GLE_CG_PER_CU=1" --tag c5 > $O/c5exp.jsonl 2> $O/c5exp.err || { echo "c5exp failed"; tail -20 $O/c5exp.err; exit 1; }
python3 -c "
import json
for l in open('$O/c5exp.jsonl'):
    d=json.loads(l)
    print('%-22s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], d['finite'])
"
