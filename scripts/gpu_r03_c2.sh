#!/bin/bash
# C2 (1 trajectory, direct ladder) kernel evidence: rocprofv3 kernel trace + stats of the C2 bench
# command, FETCH_SIZE / WRITE_SIZE passes over the direct contraction kernel (bench.py's roofline
# window), then the C2 bench line again with that traffic file.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r03c2}
mkdir -p $O/prof $O/pmc
B="bench.py --config C2 --ntraj 1 --steps 256 --warmup 32 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $B > $O/prof/bench.json 2> $O/prof/bench.err || { echo "prof failed"; tail -20 $O/prof/bench.err; exit 1; }
N=$(python3 -c "import json;print(json.load(open('$O/prof/bench.json'))['roofline']['launches'])")
python3 scripts/trace_summary.py $O/prof/run_kernel_trace.csv --steps --gaps --last contract_kernel $N --skip $N > $O/prof/summary.txt
tail -8 $O/prof/summary.txt
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc/$c -o run -- \
    python3 $B > $O/pmc/$c.json 2> $O/pmc/$c.err || { echo "pmc $c failed"; tail -20 $O/pmc/$c.err; exit 1; }
done
python3 scripts/pmc_summary.py $O/pmc $O/pmc/traffic_contract.json --kernel contract_kernel --config C2 --ntraj 1 --far-mode direct
timeout -k 10 300 python3 bench.py --config C2 --ntraj 1 --steps 256 --warmup 32 --traffic-json $O/pmc/traffic_contract.json > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench c2 failed"; tail -30 $O/bench_c2.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench_c2.json')); r=d['roofline']
print('C2 %.0f steps/s  %.1f us/step  %s %.2f frac %.3f traffic %s alg %s' % (d['value'], d['ms_per_step']*1e3, r['unit'], r['achieved'], r['frac'], r['traffic'], r['algorithmic_bytes_per_launch']))
"
