#!/bin/bash
# chain operand attribution (timing only, wrong results): CH_DBG=1 no A loads, 2 no X loads, 4 no X
# loads in the 64-column near-field tiles; current vs r03 library; C3, 3 interleaved rounds
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r04dbg}
mkdir -p $O
: > $O/libs.jsonl
for r in 1 2 3; do
  for lib in exp r03 dbg1 dbg2 dbg4; do
    SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_$lib.so timeout -k 10 200 python scripts/exp_time.py --tag $lib --chainprof 1 >> $O/libs.jsonl 2>> $O/libs.err || { echo "lib $lib failed"; tail -5 $O/libs.err; exit 1; }
  done
done
python3 - $O/libs.jsonl <<'PY'
import json, sys, collections
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l)
    agg[d["tag"]].append((d["ms_per_step"] * 1e3, d["short_ms_per_step"] * 1e3, d.get("chain_us_per_step", 0)))
for v, xs in agg.items():
    print("%-6s long %s | short %s | chain %s" % (v, " ".join("%.2f" % x[0] for x in xs), " ".join("%.2f" % x[1] for x in xs), " ".join("%.2f" % x[2] for x in xs)))
PY
