#!/bin/bash
# Parity suite on the current code, then same-box A/B of the chain register fix (no spills) against
# the previous chain build (libhipgle_old.so: experiment build of the parent commit), 3 interleaved
# rounds in separate processes, then the transform pieces on / off (GLE_FFT_CHUNK=0) in one process.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ab1
mkdir -p $O
if [ -z "$NOTESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
fi
: > $O/ab.jsonl
for r in 1 2 3; do
  for lib in old exp; do
    SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_$lib.so timeout -k 10 240 python scripts/exp_time.py --chainprof 1 --steps 512 --short-reps 8 --tag $lib >> $O/ab.jsonl 2>> $O/ab.err || { echo "ab $lib failed"; tail -20 $O/ab.err; exit 1; }
  done
done
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 400 python scripts/exp_time.py --steps 512 --short-reps 16 --rounds 2 --variants "GLE_FFT_CHUNK=0;GLE_FFT_CHUNK=32" --tag fft >> $O/ab.jsonl 2>> $O/ab.err || { echo "fft ab failed"; tail -20 $O/ab.err; exit 1; }
python3 -c "
import json, statistics as st
for l in open('$O/ab.jsonl'):
    d=json.loads(l); r=d['short_reps_ms']
    print('%-4s %-18s'%(d['tag'], d['variant']), 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'reps mean %.4f max %.4f'%(st.mean(r), max(r)) if r else '', 'chain us/step %.1f'%d.get('chain_us_per_step',0))
"
