#!/bin/bash
# (1) C3 window-length sweep (median of 9 sync-bracketed windows per length): per-window fixed cost
# vs per-step cost; (2) C2 (one trajectory, direct far field) at larger direct block lengths.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03c2w
mkdir -p $O
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 300 python scripts/exp_time.py --steps 512 --windows "10,20,40,80,160,320" --tag win > $O/win.jsonl 2> $O/win.err || { echo "win failed"; tail -20 $O/win.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/win.jsonl').readline()); w=d['window_ms']; print('long', d['ms_per_step'], w)
import numpy as np
K=np.array([int(k) for k in w]); T=np.array([w[k] for k in w]); b,a=np.polyfit(K,T,1); print('fit: %.1f us per window + %.2f us per step'%(a*1e3,b*1e3))
"
for mb in 0 64 128 256; do
  timeout -k 10 300 python bench.py --config C2 --ntraj 1 --steps 256 --warmup 32 --no-cpu-baseline --max-block $mb > $O/c2_mb$mb.json 2> $O/c2_mb$mb.err || { echo "c2 $mb failed"; tail -20 $O/c2_mb$mb.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$O/c2_mb$mb.json')); r=d.get('roofline',{})
print('C2 max_block $mb', '%.0f steps/s'%d['value'], 'us/step %.1f'%(d['ms_per_step']*1e3), 'roof %s %.0f frac %.3f'%(r.get('unit'), r.get('achieved',0), r.get('frac',0)), [l['P'] for l in d['ladder_window']])
"
done
# (3) C3 first block length 4 (near field lags [2, 8), a direct P = 4 level beside it) vs 8
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 400 python scripts/exp_time.py --steps 512 --short-reps 8 --rounds 2 --variants "EXP_BLOCK_LEN=8;EXP_BLOCK_LEN=4;EXP_BLOCK_LEN=4,GLE_SPEC_MIN=4" --tag p0 > $O/p0.jsonl 2>> $O/win.err || { echo "p0 failed"; tail -20 $O/win.err; exit 1; }
python3 -c "
import json, statistics as st
for l in open('$O/p0.jsonl'):
    d=json.loads(l); r=d['short_reps_ms']
    print('%-32s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'reps mean %.4f max %.4f'%(st.mean(r), max(r)))
"
