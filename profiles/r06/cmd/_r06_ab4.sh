set -o pipefail
mkdir -p gpurun_out/r06/t6 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_composed.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06/t6/tests.log 2>&1 && tail -2 gpurun_out/r06/t6/tests.log && \
LIBS="base xc5" ROUNDS=3 EXPARGS="--config C2 --ntraj 1" bash scripts/gpu_evidence.sh r06/ab6_c2 ab && \
LIBS="base xc5" ROUNDS=3 bash scripts/gpu_evidence.sh r06/ab6_c3 ab
