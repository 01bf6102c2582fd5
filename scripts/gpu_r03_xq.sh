#!/bin/bash
# XCD work queue for the chain launches (GLE_XCD_QUEUE=mode, experiment build): parity tests with
# it on, then C3 timing of the grouping modes against the plan order, one process.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03xq
mkdir -p $O
L=$PWD/sclmd_amd/_lib/libhipgle_exp.so
SCLMD_AMD_LIB=$L GLE_XCD_QUEUE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_configs.py tests/test_gpu_md.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SCLMD_AMD_LIB=$L timeout -k 10 500 python scripts/exp_time.py --steps 512 --short-reps 8 --rounds 2 --variants ";GLE_XCD_QUEUE=1;GLE_XCD_QUEUE=2;GLE_XCD_QUEUE=3;GLE_DBG_NO_LADDER=1;GLE_DBG_NO_LADDER=1,GLE_XCD_QUEUE=1;GLE_DBG_NO_LADDER=1,GLE_XCD_QUEUE=3" --tag xq > $O/xq.jsonl 2> $O/xq.err || { echo "xq failed"; tail -20 $O/xq.err; exit 1; }
python3 -c "
import json, statistics as st
for l in open('$O/xq.jsonl'):
    d=json.loads(l); r=d['short_reps_ms']
    print('%-18s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'reps mean %.4f'%st.mean(r), d['finite'])
"
