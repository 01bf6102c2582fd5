#!/bin/bash
# C3 first-level block length A/B (public plan option --block-len): near field lags [1, 2 P0),
# spectral levels from P0 up; 512-step and driver 20/5 windows, 2 interleaved rounds, one box
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r04p0}
mkdir -p $O
: > $O/lines.jsonl
for r in 1 2; do
  for p0 in 8 4 16; do
    timeout -k 10 200 python bench.py --block-len $p0 --no-cpu-baseline > $O/b_${p0}_$r.json 2> $O/b_${p0}_$r.err || { echo "bench $p0 failed"; tail -20 $O/b_${p0}_$r.err; exit 1; }
    timeout -k 10 200 python bench.py --block-len $p0 --steps 20 --warmup 5 --no-cpu-baseline > $O/s_${p0}_$r.json 2> $O/s_${p0}_$r.err || { echo "bench20 $p0 failed"; tail -20 $O/s_${p0}_$r.err; exit 1; }
    python3 -c "
import json
a=json.load(open('$O/b_${p0}_$r.json')); b=json.load(open('$O/s_${p0}_$r.json'))
print(json.dumps({'p0': $p0, 'round': $r, 'long_us': a['ms_per_step']*1e3, 'short_us': b['ms_per_step']*1e3, 'long_value': a['value'], 'short_value': b['value'], 'chain_us': a['chain_roofline']['us_per_step'], 'scan': b.get('window_phase'), 'levels': [l['P'] for l in a['ladder_window']]}))" | tee -a $O/lines.jsonl
  done
done
