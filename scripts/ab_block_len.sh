set -o pipefail
O=gpurun_out/r05bl; mkdir -p $O
for r in 1 2; do
 for bl in 0 4; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --block-len $bl > $O/c3_bl${bl}_$r.json 2> $O/c3_bl${bl}_$r.err || exit 1
 done
 for bl in 0 4 16; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --config C2 --ntraj 1 --steps 256 --warmup 32 --block-len $bl > $O/c2_bl${bl}_$r.json 2> $O/c2_bl${bl}_$r.err || exit 1
 done
done
python3 - <<'PY'
import json,glob
for p in sorted(glob.glob("gpurun_out/r05bl/*.json")):
    d=json.loads([l for l in open(p) if l.startswith("{")][-1])
    print(p.split("/")[-1], "%.0f"%d["value"], "%.2f us"%(d["ms_per_step"]*1e3), "bl", d["config"]["block_len"], "chain %.1f"%d.get("chain_roofline",{}).get("us_per_step",0))
PY
