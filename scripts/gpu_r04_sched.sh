#!/bin/bash
# ladder schedule switches A/B on the driver's short window (C3; EXP_ARGS="--config C5 --ntraj 32 --steps 256" for C5): mean over the 20-step windows of
# every phase of the largest level (what bench.py's 20/5 line samples) and the 512-step window,
# variants interleaved over 3 rounds in one process
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r04sched}
mkdir -p $O
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 ${TMO:-600} python scripts/exp_time.py --rounds ${ROUNDS:-3} --phase-scan 20 $EXP_ARGS \
  --variants "${VARS:-;GLE_PIECE_SLACK=1;GLE_CG_PER_CU=2;GLE_BG_GROUP=8,64}" \
  > $O/sched.jsonl 2> $O/sched.err || { echo "exp_time failed"; tail -20 $O/sched.err; exit 1; }
python3 - $O/sched.jsonl <<'PY'
import json, sys, collections
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l)
    sc = [x for _, x in d["phase_scan"]]
    agg[d.get("variant", "")].append((d["ms_per_step"] * 1e3, 1e3 * sum(sc) / len(sc), 1e3 * max(sc)))
for v, xs in agg.items():
    print("%-22s long %s | scan mean %s | scan max %s" % (v or "default", " ".join("%.2f" % x[0] for x in xs),
          " ".join("%.2f" % x[1] for x in xs), " ".join("%.2f" % x[2] for x in xs)))
PY
