#!/bin/bash
# per-workgroup chain timelines (GLE_CHAIN_DBG stamps at step 700, chain alone: GLE_DBG_NO_LADDER)
# of the current experiment build and the no-operand-load build (CH_DBG=3), C3
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r04tl}
mkdir -p $O
for lib in ${LIBS:-exp dbg3}; do
  for v in "GLE_DBG_NO_LADDER=1" "GLE_PIECE_SLACK=0"; do
    env $v GLE_CHAIN_DBG=700 SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_$lib.so timeout -k 10 200 python scripts/exp_time.py --tag "$lib $v" --steps 256 > $O/$lib.$v.json 2> $O/$lib.$v.err || { echo "$lib $v failed"; tail -5 $O/$lib.$v.err; exit 1; }
    echo "== $lib $v"; grep "chain dbg" $O/$lib.$v.err
  done
done
