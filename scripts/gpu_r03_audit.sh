#!/bin/bash
# (1) padded-operand audit build (-DGLE_BOUNDS): the whole GPU suite with every checked load / store
# against the live allocations (gle_sync fails on a miss); (2) C5 fused-stage waves 4 vs 8 with the
# fpot launch, 3 interleaved rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03audit
mkdir -p $O
SCLMD_AMD_LIB=$PWD/sclmd_amd/_lib/libhipgle_bounds.so timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests_bounds.log 2>&1 || { echo "bounds tests failed"; grep -E "FAILED|Error|bounds" $O/gpu_tests_bounds.log | head; tail -30 $O/gpu_tests_bounds.log; exit 1; }
tail -2 $O/gpu_tests_bounds.log
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 900 python -u scripts/exp_time.py --config C5 --ntraj 32 --steps 128 --rounds 3 --variants ";GLE_CHAIN_NW=4,4,4" --tag c5nw > $O/c5nw.jsonl 2> $O/c5nw.err || { echo "c5nw failed"; tail -20 $O/c5nw.err; exit 1; }
python3 -c "
import json
for l in open('$O/c5nw.jsonl'):
    d=json.loads(l); print('%-22s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], d['finite'])
"
