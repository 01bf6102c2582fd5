#!/bin/bash
# round-4 C5 evidence on the current code (one GPU's share: 32 trajectories, coloured noise streamed):
# bench line over one period of the P = 1024 level's ... window, rocprofv3 kernel trace + stats of the
# same command, FETCH_SIZE / WRITE_SIZE PMC passes of the far-field GEMM, then the same-box CPU
# baseline.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r04c5}
mkdir -p $O/prof $O/pmc
ARGS="--config C5 --ntraj 32 --steps 256 --warmup 16"
timeout -k 10 400 python -u bench.py $ARGS --cpu-budget 20 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python3 -c "
import json
d=json.load(open('$O/bench.json')); r=d.get('roofline',{}); s=d['step_roofline']
print('C5 %.0f traj-steps/s'%d['value'], 'us/step %.1f'%(d['ms_per_step']*1e3), 'cgemm %s %.1f %s frac %.3f'%(r.get('bound'), r.get('achieved',0), r.get('unit'), r.get('frac',0)), 'launches', r.get('launches'), 'avg us %.1f'%(r.get('avg_launch_ms',0)*1e3), 'cpu', d.get('cpu_baseline',{}).get('value'))
"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py $ARGS --no-cpu-baseline > $O/prof/bench.json 2> $O/prof/bench.err || { echo "prof failed"; tail -20 $O/prof/bench.err; exit 1; }
N=$(python3 -c "import json;print(json.load(open('$O/prof/bench.json'))['roofline']['launches'])")
python3 scripts/trace_summary.py $O/prof/run_kernel_trace.csv --steps --gaps --last cgemm $N --skip $N > $O/prof/summary.txt
tail -8 $O/prof/summary.txt
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $c --output-format csv -d $O/pmc/$c -o run -- \
    python3 bench.py $ARGS --no-cpu-baseline > $O/pmc/$c.json 2> $O/pmc/$c.err || { echo "pmc $c failed"; tail -20 $O/pmc/$c.err; exit 1; }
done
python3 scripts/pmc_summary.py $O/pmc $O/pmc/traffic.json --kernel cgemm_kernel --config C5 --ntraj 32
