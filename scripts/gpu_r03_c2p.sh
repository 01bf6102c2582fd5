#!/bin/bash
# Direct ladder levels issued as item-chunk pieces: parity (direct-mode tests), then C2 (one
# trajectory) at direct block caps 64 / 128 / 256 with pieces off (1), default, 4 and 8.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03c2p
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_md.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
V=""
for mb in 64 128 256; do V="$V;EXP_MAX_BLOCK=$mb,GLE_DIRECT_PIECES=1;EXP_MAX_BLOCK=$mb;EXP_MAX_BLOCK=$mb,GLE_DIRECT_PIECES=4;EXP_MAX_BLOCK=$mb,GLE_DIRECT_PIECES=8"; done
V=${V#;}
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 600 python scripts/exp_time.py --config C2 --ntraj 1 --steps 512 --short-reps 4 --rounds 2 --variants "$V" --tag c2 > $O/c2.jsonl 2> $O/c2.err || { echo "c2 failed"; tail -20 $O/c2.err; exit 1; }
python3 -c "
import json, statistics as st
for l in open('$O/c2.jsonl'):
    d=json.loads(l); r=d['short_reps_ms']
    print('%-40s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'reps mean %.4f'%st.mean(r), d['finite'])
"
