#!/bin/bash
# C3 sanity bench, then a C5 throughput run (1000 atoms, ml = 4096, 2 phonon + 1 biased electron
# bath, 32 trajectories = one GPU's share of the 256-trajectory ensemble), white noise injected
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 160 --warmup 32 > gpurun_out/c3q.json 2> gpurun_out/c3q.err || { tail -20 gpurun_out/c3q.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/c3q.json'));print('C3', round(d['value']), round(d['ms_per_step']*1e3,1),'us/step')"
timeout -k 10 900 python -u bench.py --config C5 --ntraj 32 --noise white --no-cpu-baseline "$@" > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail -30 gpurun_out/c5.err; exit 1; }
grep "\[bench\]" gpurun_out/c5.err
cat gpurun_out/c5.json
