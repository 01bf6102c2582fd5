set -o pipefail
mkdir -p gpurun_out/r06/t8 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_composed.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06/t8/tests.log 2>&1 && tail -2 gpurun_out/r06/t8/tests.log && \
LIBS="base xc5 xl1" ROUNDS=3 bash scripts/gpu_evidence.sh r06/ab8_c3 ab && \
LIBS="base xl1" ROUNDS=2 EXPARGS="--config C2 --ntraj 1" bash scripts/gpu_evidence.sh r06/ab8_c2 ab
