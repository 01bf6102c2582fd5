#!/bin/bash
# MFMA-pipe utilisation: one counters-only rocprofv3 pass over a bench run
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/mfma
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/mfma -o run -- \
  python3 bench.py --no-cpu-baseline --steps 512 --warmup 64 > gpurun_out/mfma/bench.json 2> gpurun_out/mfma/bench.err || { echo "pmc failed"; tail -20 gpurun_out/mfma/bench.err; exit 1; }
N=$(python3 -c "import json;print(json.load(open('gpurun_out/mfma/bench.json'))['roofline']['launches'])")
F=$(ls gpurun_out/mfma/*counter_collection.csv | head -1)
python3 scripts/mfma_summary.py "$F" $N gpurun_out/mfma/mfma_util.json
