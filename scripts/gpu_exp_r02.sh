#!/bin/bash
# round-2 chain experiments: parity of the release library first, then timing variants
# (experiment builds, GLE_* switches) -> gpurun_out/exp.jsonl.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_full_configs.py} -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/exp_tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/exp_tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 gpurun_out/exp_tests.log
: > gpurun_out/exp.jsonl
run() {  # lib, env..., tag
  local lib=$1; shift
  env SCLMD_AMD_LIB=sclmd_amd/_lib/$lib "$@" timeout -k 10 120 python scripts/exp_time.py --tag "$lib $*" >> gpurun_out/exp.jsonl 2>> gpurun_out/exp.err || { echo "exp failed: $lib $*"; tail -20 gpurun_out/exp.err; exit 1; }
  tail -1 gpurun_out/exp.jsonl
}
# VARIANTS: space-separated lib:ENV=V:ENV=V specs
for spec in ${VARIANTS:-libhipgle_exp.so:GLE_CHAIN_NW=4,8,4 libhipgle_db.so:GLE_CHAIN_NW=4,8,4}; do
  set -- ${spec//:/ }
  run "$@" || exit 1
  run "$@" GLE_DBG_NO_LADDER=1 || exit 1
done
