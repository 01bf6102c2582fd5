#!/bin/bash
# HBM traffic of the roofline kernel (bench.py roofline.kernel): one rocprofv3 pass per counter
# (FETCH_SIZE, WRITE_SIZE), counters only (no other trace domains), short bench runs; the summary
# keeps the dispatches of the timed region (the last roofline.launches of the kernel).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
K=${PMC_KERNEL:-cgemm_kernel}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc/$c -o run -- \
    python3 bench.py --no-cpu-baseline --steps 512 --warmup 64 "$@" > gpurun_out/pmc/$c.json 2> gpurun_out/pmc/$c.err || { echo "pmc $c failed"; tail -20 gpurun_out/pmc/$c.err; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc gpurun_out/pmc/traffic.json --kernel "$K"
