#!/bin/bash
# round-3 first GPU pass: the new tests (large-bath plan vs oracle, RCCL paths, stream abort,
# symmetric dyn rule) first, then the whole parity suite, then the driver-style bench line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
NEW="tests/test_gpu_full_configs.py tests/test_gpu_rccl.py tests/test_gpu_noise_stream.py tests/test_gpu_dyn.py"
timeout -k 10 600 python -u -m pytest $NEW -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r03/new_tests.log 2>&1
rc=$?
tail -25 gpurun_out/r03/new_tests.log
[ $rc -eq 0 ] || { echo "new tests rc=$rc"; exit 1; }
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r03/gpu_tests.log 2>&1 || { echo "suite failed"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03/gpu_tests.log | tail -20; exit 1; }
tail -3 gpurun_out/r03/gpu_tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03/bench_20.json 2> gpurun_out/r03/bench_20.err || { echo "bench20 failed"; tail -30 gpurun_out/r03/bench_20.err; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/r03/bench_20.json')); r=d.get('roofline',{}); c=d.get('chain_roofline',{})
print('%.0f traj-steps/s'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'roof %.3f'%r.get('frac',0), 'chain us/step %.1f frac %.3f'%(c.get('us_per_step',0), c.get('frac',0)), d['window_phase'])
"
