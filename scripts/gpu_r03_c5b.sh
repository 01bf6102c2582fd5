#!/bin/bash
# large-bath plan with the fpot launch: its oracle tests, then C5 plan variants (32-column DOF
# tiles, 4-wave fused tiles) in one process.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03c5b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_configs.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 900 python -u scripts/exp_time.py --config C5 --ntraj 32 --steps 128 --rounds 2 --variants ";GLE_CHAIN_DRN=2;GLE_CHAIN_NW=4,4,4" --tag c5 > $O/c5.jsonl 2> $O/c5.err || { echo "c5 failed"; tail -20 $O/c5.err; exit 1; }
python3 -c "
import json
for l in open('$O/c5.jsonl'):
    d=json.loads(l); print('%-22s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], d['finite'])
"
