#!/bin/bash
# HBM traffic of the dominant kernel: one rocprofv3 pass per counter (FETCH_SIZE, WRITE_SIZE),
# counters only (no other trace domains), short bench runs.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc/$c -o run -- \
    python3 bench.py --no-cpu-baseline --steps 24 --warmup 4 "$@" > gpurun_out/pmc/$c.json 2> gpurun_out/pmc/$c.err || { echo "pmc $c failed"; tail -20 gpurun_out/pmc/$c.err; exit 1; }
done
find gpurun_out/pmc -name "*.csv" | head
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/calib -o run -- ./tools/peak_probe > gpurun_out/pmc/calib.json 2>&1 || exit 1
