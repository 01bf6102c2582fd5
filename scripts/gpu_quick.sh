#!/bin/bash
# one short bench (no CPU baseline); stderr shows the host enqueue time
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/quick.json 2> gpurun_out/quick.err || { tail -20 gpurun_out/quick.err; exit 1; }
grep "\[bench\]" gpurun_out/quick.err
python3 -c "import json;d=json.load(open('gpurun_out/quick.json'));print(round(d['value']), round(d['ms_per_step']*1e3,1),'us/step', d['roofline']['frac'])"
