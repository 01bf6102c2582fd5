#!/bin/bash
# C3 chain waves per workgroup without register spills: A / fused stage 4/4 (plan) vs 4/8, 8/4, 8/8.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03nw
mkdir -p $O
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 600 python scripts/exp_time.py --steps 512 --short-reps 6 --rounds 3 --variants ";GLE_CHAIN_NW=4,8,4;GLE_CHAIN_NW=8,4,4;GLE_CHAIN_NW=8,8,4" --tag nw > $O/nw.jsonl 2> $O/nw.err || { echo "nw failed"; tail -20 $O/nw.err; exit 1; }
python3 -c "
import json, statistics as st
for l in open('$O/nw.jsonl'):
    d=json.loads(l); r=d['short_reps_ms']
    print('%-20s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'reps mean %.4f'%st.mean(r), d['finite'])
"
# near-field partial slots 16 (plan) vs 32 / 48 (shorter near-field tiles), separate processes
: > $O/np.jsonl
for r in 1 2; do
  for lib in exp np32 np48; do
    SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_$lib.so timeout -k 10 240 python scripts/exp_time.py --steps 512 --short-reps 6 --tag $lib >> $O/np.jsonl 2>> $O/np.err || { echo "$lib failed"; tail -20 $O/np.err; exit 1; }
  done
done
python3 -c "
import json, statistics as st
for l in open('$O/np.jsonl'):
    d=json.loads(l); r=d['short_reps_ms']
    print('%-6s'%d['tag'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'reps mean %.4f'%st.mean(r), d['finite'])
"
