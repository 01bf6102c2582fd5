#!/bin/bash
# fused far-field schedule: parity (the spectral-plan tests first), then bench lines, then an A/B of
# fused vs background schedule in one process (experiment build).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 400 python -u -m pytest tests/test_gpu_full_configs.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r03/fused_full.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error" gpurun_out/r03/fused_full.log | tail -15; [ $rc -eq 0 ] || { tail -50 gpurun_out/r03/fused_full.log; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03/fused_b20.json 2> gpurun_out/r03/fused_b20.err || { echo "bench20 failed"; tail -30 gpurun_out/r03/fused_b20.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03/fused_b512.json 2> gpurun_out/r03/fused_b512.err || { echo "bench512 failed"; tail -30 gpurun_out/r03/fused_b512.err; exit 1; }
python3 -c "
import json
for f in ['fused_b20','fused_b512']:
    d=json.load(open('gpurun_out/r03/%s.json'%f)); r=d.get('roofline',{})
    print(f, '%.0f traj-steps/s'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'roof %.3f %s'%(r.get('frac',0), r.get('us_per_step')), d['window_phase'], d['ladder_window'])
"
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 400 python scripts/exp_time.py --variants "GLE_FAR_AFRAC=0.5;GLE_FAR_BG=1;GLE_FAR_AFRAC=0.7;GLE_FAR_AFRAC=0.3" --rounds 2 --short-reps 4 > gpurun_out/r03/fused_ab.jsonl 2> gpurun_out/r03/fused_ab.err || { echo "ab failed"; tail -20 gpurun_out/r03/fused_ab.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r03/fused_ab.jsonl'):
    d=json.loads(l); print(d['variant'], d['round'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], d['short_reps_ms'])
"
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r03/fused_suite.log 2>&1 || { echo "suite failed"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03/fused_suite.log | tail -20; exit 1; }
tail -2 gpurun_out/r03/fused_suite.log
