#!/bin/bash
# The fpot launch variant of the fused velocity stage (GLE_BC_FPOT=1, experiment build): the whole
# GPU parity suite on it, then C3 and C5 timing against the default plan in one process each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03fpot
mkdir -p $O
if [ -z "$NOTESTS" ]; then
SCLMD_AMD_LIB=$PWD/sclmd_amd/_lib/libhipgle_exp.so GLE_BC_FPOT=1 timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/gpu_tests.log | head; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
fi
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 400 python scripts/exp_time.py --steps 512 --short-reps 8 --rounds 3 --variants ";GLE_BC_FPOT=1" --tag c3 > $O/c3.jsonl 2> $O/c3.err || { echo "c3 failed"; tail -20 $O/c3.err; exit 1; }
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 600 python scripts/exp_time.py --config C5 --ntraj 32 --steps 128 --rounds 2 --variants ";GLE_BC_FPOT=1" --tag c5 > $O/c5.jsonl 2> $O/c5.err || { echo "c5 failed"; tail -20 $O/c5.err; exit 1; }
python3 -c "
import json, statistics as st
for f in ['c3','c5']:
    for l in open('$O/%s.jsonl'%f):
        d=json.loads(l); r=d['short_reps_ms']
        print(f, '%-16s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'reps mean %.4f'%st.mean(r) if r else '', d['finite'])
"
