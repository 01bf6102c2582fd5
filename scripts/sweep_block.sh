#!/bin/bash
# sweep far-field partition length (block_len) x mid-level block (mid_len) at C3
set -o pipefail
mkdir -p gpurun_out
for cfg in "64 8" "64 16" "128 8" "128 16" "96 8"; do
  set -- $cfg
  timeout -k 10 600 python bench.py --no-cpu-baseline --steps 256 --warmup 64 --block-len $1 --mid-len $2 > gpurun_out/sweep_$1_$2.json 2> gpurun_out/sweep_$1_$2.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/sweep_$1_$2.json')); print('$1 $2', round(d['value']), round(d['ms_per_step'],4))"
done
