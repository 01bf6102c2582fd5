#!/bin/bash
# Per-window fixed cost (fit of sync-bracketed window time vs length) with the ladder on / off, the
# background streams at the main stream's priority, a wider piece slack.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03win2
mkdir -p $O
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 600 python scripts/exp_time.py --steps 512 --windows "10,20,40,80,160" --window-reps 7 --variants ";GLE_DBG_NO_LADDER=1;GLE_BG_SAMEPRIO=1;GLE_PIECE_SLACK=2" --tag win2 > $O/win2.jsonl 2> $O/win2.err || { echo "win2 failed"; tail -20 $O/win2.err; exit 1; }
python3 -c "
import json
import numpy as np
for l in open('$O/win2.jsonl'):
    d=json.loads(l); w=d['window_ms']
    K=np.array([int(k) for k in w]); T=np.array([w[k] for k in w]); b,a=np.polyfit(K,T,1)
    print('%-22s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'fit %.1f us/window + %.2f us/step'%(a*1e3,b*1e3), 'w20 %.1f us/step'%(w['20']/20*1e3))
"
