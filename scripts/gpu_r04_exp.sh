#!/bin/bash
# round-4 experiments (experiment library, GLE_* switches, A/B interleaved in one process per config)
set -o pipefail
OUT=gpurun_out/${1:-r04exp}
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
EXP="SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so"
env SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so GLE_CHAIN_DBG=1000 timeout -k 10 300 python scripts/exp_time.py --tag dbg \
  --variants ";GLE_CH_ORDER=1;GLE_RAW_RN=2" > $OUT/chaindbg.jsonl 2> $OUT/chaindbg.err || { tail -20 $OUT/chaindbg.err; exit 1; }
grep "chain dbg" $OUT/chaindbg.err
env SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 600 python scripts/exp_time.py --tag c3 --rounds 2 --short-reps 8 \
  --variants "${C3VARIANTS:-;GLE_CH_ORDER=1;GLE_RAW_RN=2;GLE_CH_ORDER=1,GLE_RAW_RN=2;GLE_CG_UNITS=0}" > $OUT/exp_c3.jsonl 2> $OUT/exp_c3.err || { tail -20 $OUT/exp_c3.err; exit 1; }
python3 - $OUT/exp_c3.jsonl <<'PY'
import json, sys, collections
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l)
    agg[d["variant"]].append((d["ms_per_step"] * 1e3, d["short_ms_per_step"] * 1e3, sum(d["short_reps_ms"]) / max(1, len(d["short_reps_ms"])) * 1e3))
for v, xs in agg.items():
    print("%-40s long %s | short %s | reps %s" % (v or "(default)", " ".join("%.2f" % x[0] for x in xs),
          " ".join("%.2f" % x[1] for x in xs), " ".join("%.2f" % x[2] for x in xs)))
PY
