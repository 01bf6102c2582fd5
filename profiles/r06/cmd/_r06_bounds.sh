set -o pipefail
mkdir -p gpurun_out/r06/bounds
SCLMD_AMD_LIB=$PWD/sclmd_amd/_lib/libhipgle_bounds.so timeout -k 10 900 python -u -m pytest tests/test_gpu_composed.py tests/test_gpu_parity.py tests/test_gpu_full_configs.py tests/test_gpu_md.py tests/test_gpu_noise_stream.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/bounds/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r06/bounds/tests.log; exit $rc
