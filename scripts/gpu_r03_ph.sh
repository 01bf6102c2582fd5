#!/bin/bash
# (1) per-phase 20-step window times over the largest level's period at C3 (which boundaries make
# the slow windows); (2) C5 far-field chunk sizes (workgroups per CU per GEMM chunk: 1 / 2 / 4).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ph
mkdir -p $O
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 300 python scripts/exp_time.py --steps 512 --phase-scan 20 --tag ph > $O/ph.jsonl 2> $O/ph.err || { echo "ph failed"; tail -20 $O/ph.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/ph.jsonl').readline()); sc=sorted(d['phase_scan'])
print('long', d['ms_per_step']); print(' '.join('%d:%.1f'%(p, m*1e3) for p, m in sc))
"
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 900 python -u scripts/exp_time.py --config C5 --ntraj 32 --steps 256 --rounds 2 --variants ";GLE_CG_PER_CU=1;GLE_CG_PER_CU=4" --tag c5cpc > $O/c5cpc.jsonl 2> $O/c5cpc.err || { echo "c5cpc failed"; tail -20 $O/c5cpc.err; exit 1; }
python3 -c "
import json
for l in open('$O/c5cpc.jsonl'):
    d=json.loads(l); print('%-20s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], d['finite'])
"
