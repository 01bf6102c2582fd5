#!/bin/bash
# Where do the chain's waves wait?  SQ wave-state counters, TA busy and L2 hit / miss per dispatch
# (one counter group per pass, counters only), C3 exp_time run of the release library.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03sq
mkdir -p $O
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM" "TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 scripts/exp_time.py --steps 512 > $O/p$i.json 2> $O/p$i.err || { echo "pass $i failed"; tail -5 $O/p$i.err; exit 1; }
done
python3 - <<PY
import csv, collections, glob
for i in (1,2,3):
    rows=list(csv.DictReader(open(glob.glob('$O/p%d/*counter_collection.csv'%i)[0])))
    agg=collections.defaultdict(lambda: collections.defaultdict(float)); cnt=collections.defaultdict(set)
    for r in rows:
        k=r['Kernel_Name']
        kind='A' if 'chain_kernel<0' in k else ('BC' if 'chain_kernel<3' in k else ('cgemm' if 'cgemm' in k else None))
        if not kind: continue
        agg[kind][r['Counter_Name']]+=float(r['Counter_Value']); cnt[kind].add(r.get('Dispatch_Id'))
    for kind in agg:
        n=len(cnt[kind]); print('pass',i,kind,'dispatches',n, {c: round(v/n,1) for c,v in agg[kind].items()})
PY
