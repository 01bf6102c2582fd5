set -o pipefail
mkdir -p gpurun_out/r06/t2
timeout -k 10 300 python -u -m pytest tests/test_gpu_composed.py tests/test_gpu_noise_stream.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r06/t2/composed.log 2>&1 && tail -3 gpurun_out/r06/t2/composed.log && bash scripts/gpu_evidence.sh r06/t2 tests lines
