#!/bin/bash
# large-bath plan with 4-workgroup-per-CU far-field chunks: its oracle tests, then the C5 bench line
# over a full 256-step period.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03c5f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_configs.py tests/test_gpu_noise_stream.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench.py --config C5 --ntraj 32 --steps 256 --warmup 16 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { echo "bench c5 failed"; tail -30 $O/bench_c5.err; exit 1; }
python3 -c "
import json
d=json.load(open('$O/bench_c5.json')); r=d.get('roofline',{})
print('C5 %.0f traj-steps/s'%d['value'], 'us/step %.1f'%(d['ms_per_step']*1e3), 'cgemm %s %.1f frac %.3f'%(r.get('unit'), r.get('achieved',0), r.get('frac',0)), d['config'])
"
