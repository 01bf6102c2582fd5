#!/bin/bash
# chain latency floor (timing only, wrong results): CH_DBG=3 removes every A and X operand load of
# the chain's products, so a batch costs its MFMAs only; with and without the ladder
# (GLE_DBG_NO_LADDER: the chain alone).  C3, 2 interleaved rounds.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r04dbg3}
mkdir -p $O
: > $O/libs.jsonl
for r in 1 2; do
  for lib in exp dbg3; do
    for v in "" "GLE_DBG_NO_LADDER=1"; do
      env $v SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_$lib.so timeout -k 10 200 python scripts/exp_time.py --tag "$lib $v" --chainprof 1 >> $O/libs.jsonl 2>> $O/libs.err || { echo "lib $lib $v failed"; tail -5 $O/libs.err; exit 1; }
    done
  done
done
python3 - $O/libs.jsonl <<'PY'
import json, sys, collections
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l)
    agg[d["tag"]].append((d["ms_per_step"] * 1e3, d["short_ms_per_step"] * 1e3, d.get("chain_us_per_step", 0)))
for v, xs in agg.items():
    print("%-30s long %s | short %s | chain %s" % (v, " ".join("%.2f" % x[0] for x in xs), " ".join("%.2f" % x[1] for x in xs), " ".join("%.2f" % x[2] for x in xs)))
PY
