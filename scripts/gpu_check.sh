#!/bin/bash
# quick state check: GPU parity suite + default bench line.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/bench.json')); r=d.get('roofline',{}); s=d['step_roofline']
print('%.0f traj-steps/s'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'roof %.3f'%r.get('frac',0), 'step TF %.1f'%s['achieved_tflops'])
"
