#!/bin/bash
# round-2 evidence run: parity suite -> bench windows (driver's 20/5, default 512/64, C2) ->
# rocprofv3 kernel trace + stats of the default bench command.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
T=${TESTS:-tests}
timeout -k 10 900 python -u -m pytest $T -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_20.json 2> gpurun_out/bench_20.err || { echo "bench20 failed"; tail -30 gpurun_out/bench_20.err; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
timeout -k 10 300 python bench.py --config C2 --ntraj 1 --steps 256 --warmup 32 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo "bench c2 failed"; tail -30 gpurun_out/bench_c2.err; exit 1; }
python3 -c "
import json
for f in ['bench_20','bench','bench_c2']:
    d=json.load(open('gpurun_out/%s.json'%f)); r=d.get('roofline',{}); s=d['step_roofline']
    print(f, '%.0f traj-steps/s'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'roof %.3f'%r.get('frac',0), 'step TF %.1f'%s['achieved_tflops'], 'GB/s %.0f'%s['achieved_gbs'], d['ladder_window'])
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 bench.py --no-cpu-baseline > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err || { echo "prof failed"; tail -20 gpurun_out/prof/bench.err; exit 1; }
N=$(python3 -c "import json;print(json.load(open('gpurun_out/prof/bench.json'))['roofline']['launches'])")
python3 scripts/trace_summary.py gpurun_out/prof/run_kernel_trace.csv --steps --gaps --last cgemm $N --skip $N > gpurun_out/prof/summary.txt
tail -12 gpurun_out/prof/summary.txt
