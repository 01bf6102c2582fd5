#!/bin/bash
# upper bounds: chain with the near-field tiles' X operand loads removed (CH_DBG=4) / all X loads
# removed (CH_DBG=2), alone and beside the ladder (timing only, wrong results)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
for r in 1 2; do
for lib in exp nox noxall; do
for v in "" "GLE_DBG_NO_LADDER=1"; do
env $v SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_$lib.so timeout -k 10 200 python scripts/exp_time.py --steps 512 --tag $lib > gpurun_out/r03/x_${lib}.json 2>/dev/null || { echo "lib $lib failed"; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/r03/x_$lib.json').read()); print('$lib', '$v', 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'])
"
done; done; done
