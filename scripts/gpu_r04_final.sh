#!/bin/bash
# round-4 evidence on the final code: GPU suite -> bench lines (C3 driver 20/5, C3 512, C2, C5 32) ->
# rocprofv3 kernel trace + stats of the C3 bench -> FETCH_SIZE / WRITE_SIZE passes (cgemm roofline
# window and chain window).  Stops at the first failure.  SKIP_TESTS=1 skips the suite.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r04final}
mkdir -p $O/prof $O/pmc
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
fi
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20.json 2> $O/bench_20.err || { echo "bench20 failed"; tail -30 $O/bench_20.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
timeout -k 10 300 python bench.py --config C2 --ntraj 1 --steps 256 --warmup 32 > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench c2 failed"; tail -30 $O/bench_c2.err; exit 1; }
python3 -c "
import json, os
for f in ['bench_20','bench','bench_c2']:
    p='$O/%s.json'%f
    if not os.path.exists(p): continue
    d=json.load(open(p)); r=d.get('roofline',{}); s=d['step_roofline']; c=d.get('chain_roofline',{})
    print(f, '%.0f traj-steps/s'%d['value'], 'us/step %.1f'%(d['ms_per_step']*1e3), 'roof %s %.1f frac %.3f traffic %s'%(r.get('unit'), r.get('achieved',0), r.get('frac',0), r.get('traffic')), 'chain us/step %.1f frac %.3f'%(c.get('us_per_step',0), c.get('frac',0)), 'cpu', (d.get('cpu_baseline') or {}).get('value'), d.get('window_phase'))
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --no-cpu-baseline > $O/prof/bench.json 2> $O/prof/bench.err || { echo "prof failed"; tail -20 $O/prof/bench.err; exit 1; }
N=$(python3 -c "import json;print(json.load(open('$O/prof/bench.json'))['roofline']['launches'])")
python3 scripts/trace_summary.py $O/prof/run_kernel_trace.csv --steps --gaps --last cgemm $N --skip $N > $O/prof/summary.txt
tail -6 $O/prof/summary.txt
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc/$c -o run -- \
    python3 bench.py --no-cpu-baseline > $O/pmc/$c.json 2> $O/pmc/$c.err || { echo "pmc $c failed"; tail -20 $O/pmc/$c.err; exit 1; }
done
python3 scripts/pmc_summary.py $O/pmc $O/pmc/traffic_cgemm.json --kernel cgemm_kernel --config C3 --ntraj 64
python3 scripts/pmc_summary.py $O/pmc $O/pmc/traffic_chain.json --kernel chain_kernel --config C3 --ntraj 64 --last 1024 --skip-chain-window 0
