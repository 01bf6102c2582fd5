#!/bin/bash
# round-3 evidence run: parity suite -> bench windows (driver's 20/5, default 512/64, C2) ->
# rocprofv3 kernel trace + stats of the default bench command.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ev
mkdir -p $O/prof
T=${TESTS:-tests}
if [ -z "$NOTESTS" ]; then
timeout -k 10 900 python -u -m pytest $T -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
fi
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20.json 2> $O/bench_20.err || { echo "bench20 failed"; tail -30 $O/bench_20.err; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
timeout -k 10 300 python bench.py --config C2 --ntraj 1 --steps 256 --warmup 32 > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench c2 failed"; tail -30 $O/bench_c2.err; exit 1; }
python3 -c "
import json
for f in ['bench_20','bench','bench_c2']:
    d=json.load(open('$O/%s.json'%f)); r=d.get('roofline',{}); s=d['step_roofline']; c=d.get('chain_roofline',{})
    print(f, '%.0f traj-steps/s'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'roof %.3f'%r.get('frac',0), 'chain us/step %.1f frac %.3f'%(c.get('us_per_step',0), c.get('frac',0)), 'step TF %.1f'%s['achieved_tflops'], d.get('window_phase'))
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --no-cpu-baseline > $O/prof/bench.json 2> $O/prof/bench.err || { echo "prof failed"; tail -20 $O/prof/bench.err; exit 1; }
N=$(python3 -c "import json;print(json.load(open('$O/prof/bench.json'))['roofline']['launches'])")
python3 scripts/trace_summary.py $O/prof/run_kernel_trace.csv --steps --gaps --last cgemm $N --skip $N > $O/prof/summary.txt
tail -12 $O/prof/summary.txt
