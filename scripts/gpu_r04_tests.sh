#!/bin/bash
# round-4 GPU run: the new benched-shape / multi-rank tests first, then the whole GPU suite, then the
# C3 bench lines (driver's 20/5 and the 512-step window) and the C5 line
set -o pipefail
OUT=gpurun_out/${1:-r04a}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_full_configs.py::test_c2_bench_plan_b1_vs_oracle \
  tests/test_gpu_multirank.py \
  tests/test_gpu_full_configs.py::test_c5_full_shape_linearity_and_sampled_rows > $OUT/new_tests.log 2>&1 || { tail -50 $OUT/new_tests.log; exit 1; }
tail -5 $OUT/new_tests.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  --deselect tests/test_gpu_full_configs.py::test_c5_full_shape_linearity_and_sampled_rows > $OUT/gpu_tests.log 2>&1 || { tail -50 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_20.json 2> $OUT/bench_20.err || exit 1
cut -c1-300 $OUT/bench_20.json
timeout -k 10 600 python3 bench.py --gpus 1 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
cut -c1-300 $OUT/bench.json
timeout -k 10 600 python3 bench.py --config C5 --ntraj 32 --steps 256 --warmup 16 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit 1
cut -c1-300 $OUT/bench_c5.json
