#!/bin/bash
# round-4 C5 experiments: far-field chunking of the two-plane items, chain timeline
set -o pipefail
OUT=gpurun_out/${1:-r04c5exp}
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
env SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so GLE_CHAIN_DBG=3000 timeout -k 10 600 python scripts/exp_time.py --tag c5 --config C5 --ntraj 32 \
  --steps 256 --short 20 --rounds 1 \
  --variants "${C5VARIANTS:-;GLE_CG_PER_CU=2;GLE_CG_PER_CU=8;GLE_CG_UNITS=0;GLE_PMAX_SPEC=256}" > $OUT/exp_c5.jsonl 2> $OUT/exp_c5.err || { tail -20 $OUT/exp_c5.err; exit 1; }
grep "chain dbg" $OUT/exp_c5.err | head -40
python3 - $OUT/exp_c5.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print("%-30s long %.1f us  short %.1f us" % (d["variant"] or "(default)", d["ms_per_step"] * 1e3, d["short_ms_per_step"] * 1e3))
PY
