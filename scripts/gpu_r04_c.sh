#!/bin/bash
# round-4 run c: C3 bench lines with the spill-free chain, then current vs r03 library A/B
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r04c}
mkdir -p $O
[ -n "$NOBENCH" ] || timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_20.json 2> $O/bench_20.err || { tail -20 $O/bench_20.err; exit 1; }
[ -n "$NOBENCH" ] || cut -c1-200 $O/bench_20.json
[ -n "$NOBENCH" ] || timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
[ -n "$NOBENCH" ] || cut -c1-200 $O/bench.json
: > $O/libs.jsonl
IFS=';' read -ra VLIST <<< "${VARS:-;GLE_WAIT_EARLY=4}"
for r in 1 2 3; do
  for lib in exp r03; do
    for v in "${VLIST[@]}"; do
      env $v SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_$lib.so timeout -k 10 200 python scripts/exp_time.py --tag "$lib $v" >> $O/libs.jsonl 2>> $O/libs.err || { echo "lib $lib failed"; tail -5 $O/libs.err; exit 1; }
    done
  done
done
python3 - $O/libs.jsonl <<'PY'
import json, sys, collections
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l)
    agg[d["tag"]].append((d["ms_per_step"] * 1e3, d["short_ms_per_step"] * 1e3))
for v, xs in agg.items():
    print("%-24s long %s | short %s" % (v, " ".join("%.2f" % x[0] for x in xs), " ".join("%.2f" % x[1] for x in xs)))
PY
