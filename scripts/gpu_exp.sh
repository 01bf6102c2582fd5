#!/bin/bash
# experiment: bench variants, one per line of the list file: "ENV=.. ENV=.. | bench args"; chain
# timeline of step 100 (GLE_CHAIN_DBG) on stderr
set -o pipefail
mkdir -p gpurun_out/exp
i=0
while IFS='|' read -r envs args; do
  i=$((i+1))
  env $envs GLE_CHAIN_DBG=100 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 160 --warmup 32 $args > gpurun_out/exp/$i.json 2> gpurun_out/exp/$i.err || { echo "fail: $envs | $args"; tail -3 gpurun_out/exp/$i.err; continue; }
  python3 -c "import json;d=json.load(open('gpurun_out/exp/$i.json'));print('[$envs |$args]', round(d['value']), 'traj-steps/s', round(d['ms_per_step']*1e3,1), 'us/step')"
  grep "chain dbg" gpurun_out/exp/$i.err | grep -v "  RAW\|  SFIN" || true
done < "${1:-scripts/exp.txt}"
