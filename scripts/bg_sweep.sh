#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for cfg in "0 8" "1 8" "1 7" "1 6" "0 6" "1 5"; do
  set -- $cfg
  GLE_BG_PRIO=$1 GLE_BG_CUFRAC=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 256 --warmup 32 > gpurun_out/bg_$1_$2.json 2> gpurun_out/bg_$1_$2.err || { echo "fail $cfg"; tail -5 gpurun_out/bg_$1_$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bg_$1_$2.json'));print('prio $1 cufrac $2', round(d['value']), round(d['ms_per_step']*1e3,1))"
done
