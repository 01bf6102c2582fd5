#!/bin/bash
# round-4 GPU run b: parity subset on the three-plane / two-plane split, C3 lines, then experiments
set -o pipefail
OUT=gpurun_out/${1:-r04b}
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_full_configs.py \
  tests/test_gpu_parity.py tests/test_gpu_md.py -m gpu \
  --deselect tests/test_gpu_full_configs.py::test_c5_full_shape_linearity_and_sampled_rows > $OUT/gpu_tests.log 2>&1 || { tail -50 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_20.json 2> $OUT/bench_20.err || exit 1
cut -c1-200 $OUT/bench_20.json
timeout -k 10 600 python3 bench.py --gpus 1 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
cut -c1-200 $OUT/bench.json
bash scripts/gpu_r04_exp.sh ${1:-r04b}
