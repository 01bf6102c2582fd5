set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gmem.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/gmem_tests.log 2>&1 || { tail -40 gpurun_out/gmem_tests.log; exit 1; }
grep -E "passed|failed|C3 device" gpurun_out/gmem_tests.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-budget 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
