#!/bin/bash
# Chain batch depth (k-steps of operand loads in flight per wave) now that the chain kernel no
# longer spills: exp (U1 = 8, U4 = 2) vs U1 = 12 / 16, U4 = 4, both; separate processes, same box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03batch
mkdir -p $O
: > $O/batch.jsonl
for r in 1 2; do
  for lib in exp u12 u16 n4 u16n4; do
    SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_$lib.so timeout -k 10 240 python scripts/exp_time.py --steps 512 --short-reps 6 --tag $lib >> $O/batch.jsonl 2>> $O/batch.err || { echo "$lib failed"; tail -20 $O/batch.err; exit 1; }
  done
done
python3 -c "
import json, statistics as st
for l in open('$O/batch.jsonl'):
    d=json.loads(l); r=d['short_reps_ms']
    print('%-6s'%d['tag'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'reps mean %.4f'%st.mean(r), d['finite'])
"
