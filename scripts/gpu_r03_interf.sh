#!/bin/bash
# Where does the ladder slow the chain down?  Timing-only variants of the far-field GEMM (experiment
# build, results invalid), one process each (GLE_CG_DBG is read once per process), same box:
#   none | 1: no K-hat loads (HBM stream off, MFMAs on) | 7: no loads, MFMAs only |
#   15: no loads, no MFMAs (the workgroups only hold their slots) | DBG_SKIP=1: no far-field GEMMs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03if
mkdir -p $O
: > $O/interf.jsonl
for v in "" "GLE_CG_DBG=1" "GLE_CG_DBG=7" "GLE_CG_DBG=15" "GLE_DBG_SKIP=1" ""; do
  env $v SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 240 python scripts/exp_time.py --chainprof 1 --steps 512 --tag "$v" >> $O/interf.jsonl 2>> $O/interf.err || { echo "variant $v failed"; tail -20 $O/interf.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/interf.jsonl'):
    d=json.loads(l); print('%-18s'%d['tag'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'chain us/step %.1f'%d.get('chain_us_per_step',0))
"
# chunk size of the far-field GEMM pieces (workgroups per CU per chunk): short-window drain
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 400 python scripts/exp_time.py --steps 512 --short-reps 16 --rounds 2 --variants "GLE_CG_PER_CU=0.5;GLE_CG_PER_CU=0.25;GLE_CG_PER_CU=1" --tag cpc >> $O/cpc.jsonl 2>> $O/interf.err || { echo "cpc failed"; tail -20 $O/interf.err; exit 1; }
python3 -c "
import json, statistics as st
for l in open('$O/cpc.jsonl'):
    d=json.loads(l); r=d['short_reps_ms']
    print('%-22s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'reps mean %.4f max %.4f'%(st.mean(r), max(r)))
"
