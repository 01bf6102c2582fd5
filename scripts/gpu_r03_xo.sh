#!/bin/bash
# Does the XCD tile order (GLE_XCD_ORDER, static blockIdx grouping) cut the chain's traffic beyond
# L2, and does the time follow?  FETCH_SIZE per chain dispatch (one counter pass per mode) and
# plain timing (one process, interleaved), experiment build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03xo
mkdir -p $O
for m in 0 1 2 3; do
  GLE_XCD_ORDER=$m SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc$m -o run -- python3 scripts/exp_time.py --steps 512 > $O/pmc$m.json 2> $O/pmc$m.err || { echo "pmc $m failed"; tail -5 $O/pmc$m.err; exit 1; }
done
python3 - <<PY
import csv
for m in range(4):
    rows=[r for r in csv.DictReader(open('$O/pmc%d/run_counter_collection.csv'%m)) if 'chain_kernel' in r['Kernel_Name']]
    rows.sort(key=lambda r:int(r.get('Dispatch_Id',0)))
    v=[float(r['Counter_Value']) for r in rows][-1024:]
    a=[float(r['Counter_Value']) for r in rows if 'chain_kernelILi0' in r['Kernel_Name']][-512:]
    b=[float(r['Counter_Value']) for r in rows if 'chain_kernelILi3' in r['Kernel_Name']][-512:]
    print('order', m, 'chain MB/launch beyond L2 %.1f (A %.1f, BC %.1f)'%(2*sum(v)/len(v)*1024/1e6, 2*sum(a)/len(a)*1024/1e6, 2*sum(b)/len(b)*1024/1e6))
PY
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 400 python scripts/exp_time.py --steps 512 --short-reps 4 --rounds 2 --variants ";GLE_XCD_ORDER=1;GLE_XCD_ORDER=2;GLE_XCD_ORDER=3" --tag xo > $O/xo.jsonl 2> $O/xo.err || { echo "xo failed"; tail -20 $O/xo.err; exit 1; }
python3 -c "
import json
for l in open('$O/xo.jsonl'):
    d=json.loads(l); print('%-18s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'])
"
