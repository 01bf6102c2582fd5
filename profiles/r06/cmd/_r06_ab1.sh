set -o pipefail
LIBS="base xo0 xo1" ROUNDS=2 EXPARGS="--config C2 --ntraj 1" bash scripts/gpu_evidence.sh r06/ab1_c2 ab && \
mkdir -p gpurun_out/r06/k1 && \
timeout -k 10 500 python -u -m pytest tests/test_gpu_full_configs.py tests/test_gpu_parity.py tests/test_gpu_gmem.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/k1/tests.log 2>&1 && tail -2 gpurun_out/r06/k1/tests.log && \
bash scripts/gpu_evidence.sh r06/k1 c5
