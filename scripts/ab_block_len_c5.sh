# C5 line at first block lengths ${BLS:-2 0} (0: the planner's choice), interleaved ${ROUNDS:-1} times
set -o pipefail
O=gpurun_out/r05bl5; mkdir -p $O
for r in $(seq 1 ${ROUNDS:-1}); do for bl in ${BLS:-2 0}; do
  timeout -k 10 400 python bench.py --config C5 --ntraj 32 --steps 256 --warmup 32 --no-cpu-baseline --block-len $bl \
    > $O/c5_bl${bl}_$r.json 2> $O/c5_bl${bl}_$r.err || exit 1
done; done
python3 - <<'PY'
import json,glob
for p in sorted(glob.glob("gpurun_out/r05bl5/*.json")):
    d=json.loads([l for l in open(p) if l.startswith("{")][-1])
    print(p.split("/")[-1], "%.0f"%d["value"], "%.2f us"%(d["ms_per_step"]*1e3), "bl", d["config"]["block_len"],
          "chain %.1f"%d.get("chain_roofline",{}).get("us_per_step",0), [l["P"] for l in d["ladder_window"]])
PY
