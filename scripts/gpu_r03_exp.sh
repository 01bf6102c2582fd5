#!/bin/bash
# Round-3 GPU experiments, one function per experiment (each wrote the profiles/r03 files named
# in DESIGN.md section 3).  Usage: bash scripts/gpu_r03_exp.sh <name> [<name> ...]
# Experiment builds: `make experiments` (GLE_* switches) and, for the compile-time variants,
# `make experiments EXPNAME=<name> EXPFLAGS=...` as noted per function.
set -o pipefail
export TMPDIR=/tmp

exp_ab1() {
# Parity suite on the current code, then same-box A/B of the chain register fix (no spills) against
# the previous chain build (libhipgle_old.so: experiment build of the parent commit), 3 interleaved
# rounds in separate processes, then the transform pieces on / off (GLE_FFT_CHUNK=0) in one process.
O=gpurun_out/r03ab1
mkdir -p $O
if [ -z "$NOTESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
fi
: > $O/ab.jsonl
for r in 1 2 3; do
  for lib in old exp; do
    SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_$lib.so timeout -k 10 240 python scripts/exp_time.py --chainprof 1 --steps 512 --short-reps 8 --tag $lib >> $O/ab.jsonl 2>> $O/ab.err || { echo "ab $lib failed"; tail -20 $O/ab.err; exit 1; }
  done
done
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 400 python scripts/exp_time.py --steps 512 --short-reps 16 --rounds 2 --variants "GLE_FFT_CHUNK=0;GLE_FFT_CHUNK=32" --tag fft >> $O/ab.jsonl 2>> $O/ab.err || { echo "fft ab failed"; tail -20 $O/ab.err; exit 1; }
python3 -c "
import json, statistics as st
for l in open('$O/ab.jsonl'):
    d=json.loads(l); r=d['short_reps_ms']
    print('%-4s %-18s'%(d['tag'], d['variant']), 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'reps mean %.4f max %.4f'%(st.mean(r), max(r)) if r else '', 'chain us/step %.1f'%d.get('chain_us_per_step',0))
"

}

exp_audit() {
# (1) padded-operand audit build (-DGLE_BOUNDS): the whole GPU suite with every checked load / store
# against the live allocations (gle_sync fails on a miss); (2) C5 fused-stage waves 4 vs 8 with the
# fpot launch, 3 interleaved rounds.
O=gpurun_out/r03audit
mkdir -p $O
SCLMD_AMD_LIB=$PWD/sclmd_amd/_lib/libhipgle_bounds.so timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests_bounds.log 2>&1 || { echo "bounds tests failed"; grep -E "FAILED|Error|bounds" $O/gpu_tests_bounds.log | head; tail -30 $O/gpu_tests_bounds.log; exit 1; }
tail -2 $O/gpu_tests_bounds.log
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 900 python -u scripts/exp_time.py --config C5 --ntraj 32 --steps 128 --rounds 3 --variants ";GLE_CHAIN_NW=4,4,4" --tag c5nw > $O/c5nw.jsonl 2> $O/c5nw.err || { echo "c5nw failed"; tail -20 $O/c5nw.err; exit 1; }
python3 -c "
import json
for l in open('$O/c5nw.jsonl'):
    d=json.loads(l); print('%-22s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], d['finite'])
"

}

exp_batch() {
# Chain batch depth (k-steps of operand loads in flight per wave) now that the chain kernel no
# longer spills: exp (U1 = 8, U4 = 2) vs U1 = 12 / 16, U4 = 4, both; separate processes, same box.
O=gpurun_out/r03batch
mkdir -p $O
: > $O/batch.jsonl
for r in 1 2; do
  for lib in exp u12 u16 n4 u16n4; do
    SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_$lib.so timeout -k 10 240 python scripts/exp_time.py --steps 512 --short-reps 6 --tag $lib >> $O/batch.jsonl 2>> $O/batch.err || { echo "$lib failed"; tail -20 $O/batch.err; exit 1; }
  done
done
python3 -c "
import json, statistics as st
for l in open('$O/batch.jsonl'):
    d=json.loads(l); r=d['short_reps_ms']
    print('%-6s'%d['tag'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'reps mean %.4f'%st.mean(r), d['finite'])
"

}

exp_c2p() {
# Direct ladder levels issued as item-chunk pieces: parity (direct-mode tests), then C2 (one
# trajectory) at direct block caps 64 / 128 / 256 with pieces off (1), default, 4 and 8.
O=gpurun_out/r03c2p
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_md.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
V=""
for mb in 64 128 256; do V="$V;EXP_MAX_BLOCK=$mb,GLE_DIRECT_PIECES=1;EXP_MAX_BLOCK=$mb;EXP_MAX_BLOCK=$mb,GLE_DIRECT_PIECES=4;EXP_MAX_BLOCK=$mb,GLE_DIRECT_PIECES=8"; done
V=${V#;}
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 600 python scripts/exp_time.py --config C2 --ntraj 1 --steps 512 --short-reps 4 --rounds 2 --variants "$V" --tag c2 > $O/c2.jsonl 2> $O/c2.err || { echo "c2 failed"; tail -20 $O/c2.err; exit 1; }
python3 -c "
import json, statistics as st
for l in open('$O/c2.jsonl'):
    d=json.loads(l); r=d['short_reps_ms']
    print('%-40s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'reps mean %.4f'%st.mean(r), d['finite'])
"

}

exp_c2w() {
# (1) C3 window-length sweep (median of 9 sync-bracketed windows per length): per-window fixed cost
# vs per-step cost; (2) C2 (one trajectory, direct far field) at larger direct block lengths.
O=gpurun_out/r03c2w
mkdir -p $O
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 300 python scripts/exp_time.py --steps 512 --windows "10,20,40,80,160,320" --tag win > $O/win.jsonl 2> $O/win.err || { echo "win failed"; tail -20 $O/win.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/win.jsonl').readline()); w=d['window_ms']; print('long', d['ms_per_step'], w)
import numpy as np
K=np.array([int(k) for k in w]); T=np.array([w[k] for k in w]); b,a=np.polyfit(K,T,1); print('fit: %.1f us per window + %.2f us per step'%(a*1e3,b*1e3))
"
for mb in 0 64 128 256; do
  timeout -k 10 300 python bench.py --config C2 --ntraj 1 --steps 256 --warmup 32 --no-cpu-baseline --max-block $mb > $O/c2_mb$mb.json 2> $O/c2_mb$mb.err || { echo "c2 $mb failed"; tail -20 $O/c2_mb$mb.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$O/c2_mb$mb.json')); r=d.get('roofline',{})
print('C2 max_block $mb', '%.0f steps/s'%d['value'], 'us/step %.1f'%(d['ms_per_step']*1e3), 'roof %s %.0f frac %.3f'%(r.get('unit'), r.get('achieved',0), r.get('frac',0)), [l['P'] for l in d['ladder_window']])
"
done
# (3) C3 first block length 4 (near field lags [2, 8), a direct P = 4 level beside it) vs 8
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 400 python scripts/exp_time.py --steps 512 --short-reps 8 --rounds 2 --variants "EXP_BLOCK_LEN=8;EXP_BLOCK_LEN=4;EXP_BLOCK_LEN=4,GLE_SPEC_MIN=4" --tag p0 > $O/p0.jsonl 2>> $O/win.err || { echo "p0 failed"; tail -20 $O/win.err; exit 1; }
python3 -c "
import json, statistics as st
for l in open('$O/p0.jsonl'):
    d=json.loads(l); r=d['short_reps_ms']
    print('%-32s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'reps mean %.4f max %.4f'%(st.mean(r), max(r)))
"

}

exp_c5b() {
# large-bath plan with the fpot launch: its oracle tests, then C5 plan variants (32-column DOF
# tiles, 4-wave fused tiles) in one process.
O=gpurun_out/r03c5b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_configs.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 900 python -u scripts/exp_time.py --config C5 --ntraj 32 --steps 128 --rounds 2 --variants ";GLE_CHAIN_DRN=2;GLE_CHAIN_NW=4,4,4" --tag c5 > $O/c5.jsonl 2> $O/c5.err || { echo "c5 failed"; tail -20 $O/c5.err; exit 1; }
python3 -c "
import json
for l in open('$O/c5.jsonl'):
    d=json.loads(l); print('%-22s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], d['finite'])
"

}

exp_c5cpc() {
# C5 far-field GEMM chunk sizes (workgroups per CU per chunk), one process, interleaved rounds.
O=gpurun_out/r03c5cpc
mkdir -p $O
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 1000 python -u scripts/exp_time.py --config C5 --ntraj 32 --steps 256 --rounds 2 --variants "GLE_CG_PER_CU=4;GLE_CG_PER_CU=8;GLE_CG_PER_CU=16;GLE_CG_PER_CU=32" --tag c5cpc > $O/c5cpc.jsonl 2> $O/c5cpc.err || { echo "c5cpc failed"; tail -20 $O/c5cpc.err; exit 1; }
python3 -c "
import json
for l in open('$O/c5cpc.jsonl'):
    d=json.loads(l); print('%-20s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], d['finite'])
"

}

exp_c5exp() {
# C5 (32 trajectories) plan variants, one process, interleaved: 32-column DOF tiles (each matrix
# fragment fetched once instead of once per 16-column tile), 4-wave fused tiles, far-field chunks.
O=gpurun_out/r03c5exp
mkdir -p $O
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 900 python -u scripts/exp_time.py --config C5 --ntraj 32 --steps 128 --short 20 --rounds 2 --variants ";GLE_CHAIN_DRN=2;GLE_CHAIN_NW=4,4,4;GLE_CG_PER_CU=1" --tag c5 > $O/c5exp.jsonl 2> $O/c5exp.err || { echo "c5exp failed"; tail -20 $O/c5exp.err; exit 1; }
python3 -c "
import json
for l in open('$O/c5exp.jsonl'):
    d=json.loads(l)
    print('%-22s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], d['finite'])
"

}

exp_c5f() {
# large-bath plan with 4-workgroup-per-CU far-field chunks: its oracle tests, then the C5 bench line
# over a full 256-step period.
O=gpurun_out/r03c5f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_configs.py tests/test_gpu_noise_stream.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench.py --config C5 --ntraj 32 --steps 256 --warmup 16 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { echo "bench c5 failed"; tail -30 $O/bench_c5.err; exit 1; }
python3 -c "
import json
d=json.load(open('$O/bench_c5.json')); r=d.get('roofline',{})
print('C5 %.0f traj-steps/s'%d['value'], 'us/step %.1f'%(d['ms_per_step']*1e3), 'cgemm %s %.1f frac %.3f'%(r.get('unit'), r.get('achieved',0), r.get('frac',0)), d['config'])
"

}

exp_c5s() {
# C5 plan knobs with the new chunking: first block length 8 vs 4 (one process), 8 k-steps per
# far-field LDS chunk (GLE_CG_KC, read once per process: its own process).
O=gpurun_out/r03c5s
mkdir -p $O
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 700 python -u scripts/exp_time.py --config C5 --ntraj 32 --steps 256 --rounds 2 --variants ";EXP_BLOCK_LEN=8" --tag c5p0 > $O/c5s.jsonl 2> $O/c5s.err || { echo "c5p0 failed"; tail -20 $O/c5s.err; exit 1; }
GLE_CG_KC=8 SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 400 python -u scripts/exp_time.py --config C5 --ntraj 32 --steps 256 --tag c5kc8 >> $O/c5s.jsonl 2>> $O/c5s.err || { echo "c5kc8 failed"; tail -20 $O/c5s.err; exit 1; }
python3 -c "
import json
for l in open('$O/c5s.jsonl'):
    d=json.loads(l); print('%-8s %-20s'%(d['tag'], d['variant']), 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], d['finite'])
"

}

exp_evidence() {
# round-3 evidence run: parity suite -> bench windows (driver's 20/5, default 512/64, C2) ->
# rocprofv3 kernel trace + stats of the default bench command.  Stops at the first failure.
O=gpurun_out/r03ev
mkdir -p $O/prof
T=${TESTS:-tests}
if [ -z "$NOTESTS" ]; then
timeout -k 10 900 python -u -m pytest $T -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
fi
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20.json 2> $O/bench_20.err || { echo "bench20 failed"; tail -30 $O/bench_20.err; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
timeout -k 10 300 python bench.py --config C2 --ntraj 1 --steps 256 --warmup 32 > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench c2 failed"; tail -30 $O/bench_c2.err; exit 1; }
python3 -c "
import json
for f in ['bench_20','bench','bench_c2']:
    d=json.load(open('$O/%s.json'%f)); r=d.get('roofline',{}); s=d['step_roofline']; c=d.get('chain_roofline',{})
    print(f, '%.0f traj-steps/s'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'roof %.3f'%r.get('frac',0), 'chain us/step %.1f frac %.3f'%(c.get('us_per_step',0), c.get('frac',0)), 'step TF %.1f'%s['achieved_tflops'], d.get('window_phase'))
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --no-cpu-baseline > $O/prof/bench.json 2> $O/prof/bench.err || { echo "prof failed"; tail -20 $O/prof/bench.err; exit 1; }
N=$(python3 -c "import json;print(json.load(open('$O/prof/bench.json'))['roofline']['launches'])")
python3 scripts/trace_summary.py $O/prof/run_kernel_trace.csv --steps --gaps --last cgemm $N --skip $N > $O/prof/summary.txt
tail -12 $O/prof/summary.txt

}

exp_fpot() {
# The fpot launch variant of the fused velocity stage (GLE_BC_FPOT=1, experiment build): the whole
# GPU parity suite on it, then C3 and C5 timing against the default plan in one process each.
O=gpurun_out/r03fpot
mkdir -p $O
if [ -z "$NOTESTS" ]; then
SCLMD_AMD_LIB=$PWD/sclmd_amd/_lib/libhipgle_exp.so GLE_BC_FPOT=1 timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/gpu_tests.log | head; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
fi
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 400 python scripts/exp_time.py --steps 512 --short-reps 8 --rounds 3 --variants ";GLE_BC_FPOT=1" --tag c3 > $O/c3.jsonl 2> $O/c3.err || { echo "c3 failed"; tail -20 $O/c3.err; exit 1; }
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 600 python scripts/exp_time.py --config C5 --ntraj 32 --steps 128 --rounds 2 --variants ";GLE_BC_FPOT=1" --tag c5 > $O/c5.jsonl 2> $O/c5.err || { echo "c5 failed"; tail -20 $O/c5.err; exit 1; }
python3 -c "
import json, statistics as st
for f in ['c3','c5']:
    for l in open('$O/%s.jsonl'%f):
        d=json.loads(l); r=d['short_reps_ms']
        print(f, '%-16s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'reps mean %.4f'%st.mean(r) if r else '', d['finite'])
"

}

exp_interf() {
# Where does the ladder slow the chain down?  Timing-only variants of the far-field GEMM (experiment
# build, results invalid), one process each (GLE_CG_DBG is read once per process), same box:
#   none | 1: no K-hat loads (HBM stream off, MFMAs on) | 7: no loads, MFMAs only |
#   15: no loads, no MFMAs (the workgroups only hold their slots) | DBG_SKIP=1: no far-field GEMMs
O=gpurun_out/r03if
mkdir -p $O
: > $O/interf.jsonl
for v in "" "GLE_CG_DBG=1" "GLE_CG_DBG=7" "GLE_CG_DBG=15" "GLE_DBG_SKIP=1" ""; do
  env $v SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 240 python scripts/exp_time.py --chainprof 1 --steps 512 --tag "$v" >> $O/interf.jsonl 2>> $O/interf.err || { echo "variant $v failed"; tail -20 $O/interf.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/interf.jsonl'):
    d=json.loads(l); print('%-18s'%d['tag'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'chain us/step %.1f'%d.get('chain_us_per_step',0))
"
# chunk size of the far-field GEMM pieces (workgroups per CU per chunk): short-window drain
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 400 python scripts/exp_time.py --steps 512 --short-reps 16 --rounds 2 --variants "GLE_CG_PER_CU=0.5;GLE_CG_PER_CU=0.25;GLE_CG_PER_CU=1" --tag cpc >> $O/cpc.jsonl 2>> $O/interf.err || { echo "cpc failed"; tail -20 $O/interf.err; exit 1; }
python3 -c "
import json, statistics as st
for l in open('$O/cpc.jsonl'):
    d=json.loads(l); r=d['short_reps_ms']
    print('%-22s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'reps mean %.4f max %.4f'%(st.mean(r), max(r)))
"

}

exp_nw() {
# C3 chain waves per workgroup without register spills: A / fused stage 4/4 (plan) vs 4/8, 8/4, 8/8.
O=gpurun_out/r03nw
mkdir -p $O
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 600 python scripts/exp_time.py --steps 512 --short-reps 6 --rounds 3 --variants ";GLE_CHAIN_NW=4,8,4;GLE_CHAIN_NW=8,4,4;GLE_CHAIN_NW=8,8,4" --tag nw > $O/nw.jsonl 2> $O/nw.err || { echo "nw failed"; tail -20 $O/nw.err; exit 1; }
python3 -c "
import json, statistics as st
for l in open('$O/nw.jsonl'):
    d=json.loads(l); r=d['short_reps_ms']
    print('%-20s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'reps mean %.4f'%st.mean(r), 'w20 %.4f'%(d['window_ms']['20']/20), d['finite'])
"
# near-field partial slots 16 (plan) vs 32 / 48 (shorter near-field tiles), separate processes
: > $O/np.jsonl
for r in 1 2; do
  for lib in exp np32 np48; do
    SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_$lib.so timeout -k 10 240 python scripts/exp_time.py --steps 512 --short-reps 6 --tag $lib >> $O/np.jsonl 2>> $O/np.err || { echo "$lib failed"; tail -20 $O/np.err; exit 1; }
  done
done
python3 -c "
import json, statistics as st
for l in open('$O/np.jsonl'):
    d=json.loads(l); r=d['short_reps_ms']
    print('%-6s'%d['tag'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'reps mean %.4f'%st.mean(r), d['finite'])
"

}

exp_ph() {
# (1) per-phase 20-step window times over the largest level's period at C3 (which boundaries make
# the slow windows); (2) C5 far-field chunk sizes (workgroups per CU per GEMM chunk: 1 / 2 / 4).
O=gpurun_out/r03ph
mkdir -p $O
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 300 python scripts/exp_time.py --steps 512 --phase-scan 20 --tag ph > $O/ph.jsonl 2> $O/ph.err || { echo "ph failed"; tail -20 $O/ph.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/ph.jsonl').readline()); sc=sorted(d['phase_scan'])
print('long', d['ms_per_step']); print(' '.join('%d:%.1f'%(p, m*1e3) for p, m in sc))
"
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 900 python -u scripts/exp_time.py --config C5 --ntraj 32 --steps 256 --rounds 2 --variants ";GLE_CG_PER_CU=1;GLE_CG_PER_CU=4" --tag c5cpc > $O/c5cpc.jsonl 2> $O/c5cpc.err || { echo "c5cpc failed"; tail -20 $O/c5cpc.err; exit 1; }
python3 -c "
import json
for l in open('$O/c5cpc.jsonl'):
    d=json.loads(l); print('%-20s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], d['finite'])
"

}

exp_win2() {
# Per-window fixed cost (fit of sync-bracketed window time vs length) with the ladder on / off, the
# background streams at the main stream's priority, a wider piece slack.
O=gpurun_out/r03win2
mkdir -p $O
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 600 python scripts/exp_time.py --steps 512 --windows "10,20,40,80,160" --window-reps 7 --variants ";GLE_DBG_NO_LADDER=1;GLE_BG_SAMEPRIO=1;GLE_PIECE_SLACK=2" --tag win2 > $O/win2.jsonl 2> $O/win2.err || { echo "win2 failed"; tail -20 $O/win2.err; exit 1; }
python3 -c "
import json
import numpy as np
for l in open('$O/win2.jsonl'):
    d=json.loads(l); w=d['window_ms']
    K=np.array([int(k) for k in w]); T=np.array([w[k] for k in w]); b,a=np.polyfit(K,T,1)
    print('%-22s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'fit %.1f us/window + %.2f us/step'%(a*1e3,b*1e3), 'w20 %.1f us/step'%(w['20']/20*1e3))
"

}

exp_xq() {
# XCD work queue for the chain launches (GLE_XCD_QUEUE=mode, experiment build): parity tests with
# it on, then C3 timing of the grouping modes against the plan order, one process.
O=gpurun_out/r03xq
mkdir -p $O
L=$PWD/sclmd_amd/_lib/libhipgle_exp.so
SCLMD_AMD_LIB=$L GLE_XCD_QUEUE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_configs.py tests/test_gpu_md.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SCLMD_AMD_LIB=$L timeout -k 10 500 python scripts/exp_time.py --steps 512 --short-reps 8 --rounds 2 --variants ";GLE_XCD_QUEUE=1;GLE_XCD_QUEUE=2;GLE_XCD_QUEUE=3;GLE_DBG_NO_LADDER=1;GLE_DBG_NO_LADDER=1,GLE_XCD_QUEUE=1;GLE_DBG_NO_LADDER=1,GLE_XCD_QUEUE=3" --tag xq > $O/xq.jsonl 2> $O/xq.err || { echo "xq failed"; tail -20 $O/xq.err; exit 1; }
python3 -c "
import json, statistics as st
for l in open('$O/xq.jsonl'):
    d=json.loads(l); r=d['short_reps_ms']
    print('%-18s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'reps mean %.4f'%st.mean(r), d['finite'])
"

}

exp_kc() {
# far-field LDS chunk of 8 k-steps (GLE_CG_KC=8, read once per process) vs 4, C3 and C5, processes
# alternating over 2 rounds
O=gpurun_out/r03kc
mkdir -p $O
: > $O/kc.jsonl
for r in 1 2; do
  for kc in 4 8; do
    GLE_CG_KC=$kc SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 240 python scripts/exp_time.py --steps 512 --short-reps 4 --tag c3kc$kc >> $O/kc.jsonl 2>> $O/kc.err || { echo "c3 kc$kc failed"; tail -20 $O/kc.err; exit 1; }
    GLE_CG_KC=$kc SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 400 python -u scripts/exp_time.py --config C5 --ntraj 32 --steps 256 --tag c5kc$kc >> $O/kc.jsonl 2>> $O/kc.err || { echo "c5 kc$kc failed"; tail -20 $O/kc.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('$O/kc.jsonl'):
  d=json.loads(l); print('%-8s'%d['tag'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], d['finite'])
"
}

exp_c3cpc() {
# C3 far-field chunk sizes beyond 1 workgroup per CU (0.25-1 were flat earlier this round)
O=gpurun_out/r03c3cpc
mkdir -p $O
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 500 python scripts/exp_time.py --steps 512 --short-reps 8 --rounds 3 --windows 20 --window-reps 9 --variants ";GLE_CG_PER_CU=1;GLE_CG_PER_CU=2;GLE_CG_PER_CU=3" --tag c3cpc > $O/c3cpc.jsonl 2> $O/c3cpc.err || { echo "c3cpc failed"; tail -20 $O/c3cpc.err; exit 1; }
python3 -c "
import json, statistics as st
for l in open('$O/c3cpc.jsonl'):
    d=json.loads(l); r=d['short_reps_ms']
    print('%-20s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'short %.4f'%d['short_ms_per_step'], 'reps mean %.4f'%st.mean(r), 'w20 %.4f'%(d['window_ms']['20']/20), d['finite'])
"
}

exp_lines() {
# bench lines after the chunk-size changes: C5 cgemm FETCH / WRITE passes (per-launch traffic for the
# new chunking), then the C3 (20/5, 512) and C5 (256-step period) lines reading the new traffic files
O=gpurun_out/r03lines
mkdir -p $O/pmc
for c in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 400 rocprofv3 --pmc $c --output-format csv -d $O/pmc/$c -o run -- python3 bench.py --config C5 --ntraj 32 --steps 256 --warmup 16 --no-cpu-baseline > $O/pmc/$c.json 2> $O/pmc/$c.err || { echo "pmc $c failed"; tail -20 $O/pmc/$c.err; exit 1; }
done
python3 scripts/pmc_summary.py $O/pmc $O/pmc/traffic_c5.json --kernel cgemm_kernel --config C5 --ntraj 32 || exit 1
cp $O/pmc/traffic_c5.json profiles/traffic_C5_32.json
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20.json 2> $O/bench_20.err || { echo "bench20 failed"; tail -30 $O/bench_20.err; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
timeout -k 10 400 python bench.py --config C5 --ntraj 32 --steps 256 --warmup 16 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { echo "bench c5 failed"; tail -30 $O/bench_c5.err; exit 1; }
python3 -c "
import json
for f in ['bench_20','bench','bench_c5']:
    d=json.load(open('$O/%s.json'%f)); r=d.get('roofline',{})
    print(f, '%.0f traj-steps/s'%d['value'], 'us/step %.1f'%(d['ms_per_step']*1e3), 'roof %s %.1f frac %.3f traffic %s algo %s'%(r.get('unit'), r.get('achieved',0), r.get('frac',0), r.get('traffic'), r.get('algorithmic_bytes_per_launch')), d.get('window_phase'))
"
}

exp_fftp() {
# transform piece size (GLE_FFT_CHUNK = P per piece) and piece cadence with the 2-per-CU GEMM chunks
O=gpurun_out/r03fftp
mkdir -p $O
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 700 python scripts/exp_time.py --steps 512 --short-reps 8 --rounds 3 --windows 20 --window-reps 9 --variants ";GLE_FFT_CHUNK=16;GLE_FFT_CHUNK=64;GLE_PIECE_STEP=2" --tag fftp > $O/fftp.jsonl 2> $O/fftp.err || { echo "fftp failed"; tail -20 $O/fftp.err; exit 1; }
python3 -c "
import json, statistics as st
for l in open('$O/fftp.jsonl'):
    d=json.loads(l); r=d['short_reps_ms']
    print('%-20s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'reps mean %.4f max %.4f'%(st.mean(r), max(r)), 'w20 %.4f'%(d['window_ms']['20']/20), d['finite'])
"
}

exp_split() {
# small spectral levels without the k-split of their products (GLE_CG_SPLIT=0), and the far-field
# items without the XCD grouping (GLE_CG_XCD=0, read once per process: its own process)
O=gpurun_out/r03split
mkdir -p $O
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 500 python scripts/exp_time.py --steps 512 --short-reps 8 --rounds 3 --windows 20 --window-reps 9 --variants ";GLE_CG_SPLIT=0" --tag split > $O/split.jsonl 2> $O/split.err || { echo "split failed"; tail -20 $O/split.err; exit 1; }
GLE_CG_XCD=0 SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 300 python scripts/exp_time.py --steps 512 --short-reps 8 --windows 20 --window-reps 9 --tag noxcd >> $O/split.jsonl 2>> $O/split.err || { echo "noxcd failed"; tail -20 $O/split.err; exit 1; }
python3 -c "
import json, statistics as st
for l in open('$O/split.jsonl'):
    d=json.loads(l); r=d['short_reps_ms']
    print('%-8s %-16s'%(d['tag'], d['variant']), 'long %.4f'%d['ms_per_step'], 'reps mean %.4f'%st.mean(r), 'w20 %.4f'%(d['window_ms']['20']/20), d['finite'])
"
}

exp_final4() {
# current code: parity suite, C3 cgemm / chain PMC passes first (traffic per launch for the current
# chunking into profiles/traffic_C3_64.json), then the C3 / C2 bench lines and the C3 kernel trace
O=gpurun_out/r03final4
mkdir -p $O/prof $O/pmc
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/gpu_tests.log | head; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for c in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc/$c -o run -- python3 bench.py --no-cpu-baseline > $O/pmc/$c.json 2> $O/pmc/$c.err || { echo "pmc $c failed"; tail -20 $O/pmc/$c.err; exit 1; }
done
python3 scripts/pmc_summary.py $O/pmc $O/pmc/traffic_cgemm.json --kernel cgemm_kernel --config C3 --ntraj 64 || exit 1
python3 scripts/pmc_summary.py $O/pmc $O/pmc/traffic_chain.json --kernel chain_kernel --config C3 --ntraj 64 --last 1024 --skip-chain-window 0 || exit 1
cp $O/pmc/traffic_cgemm.json profiles/traffic_C3_64.json
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20.json 2> $O/bench_20.err || { echo "bench20 failed"; tail -30 $O/bench_20.err; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
timeout -k 10 300 python bench.py --config C2 --ntraj 1 --steps 256 --warmup 32 > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench c2 failed"; tail -30 $O/bench_c2.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/prof/bench.json 2> $O/prof/bench.err || { echo "prof failed"; tail -20 $O/prof/bench.err; exit 1; }
N=$(python3 -c "import json;print(json.load(open('$O/prof/bench.json'))['roofline']['launches'])")
python3 scripts/trace_summary.py $O/prof/run_kernel_trace.csv --steps --gaps --last cgemm $N --skip $N > $O/prof/summary.txt
tail -4 $O/prof/summary.txt
python3 -c "
import json
for f in ['bench_20','bench','bench_c2']:
    d=json.load(open('$O/%s.json'%f)); r=d.get('roofline',{}); c=d.get('chain_roofline',{})
    print(f, '%.0f traj-steps/s'%d['value'], 'us/step %.1f'%(d['ms_per_step']*1e3), 'roof %s %.1f frac %.3f traffic %s algo %s'%(r.get('unit'), r.get('achieved',0), r.get('frac',0), r.get('traffic'), r.get('algorithmic_bytes_per_launch')), 'chain %.1f frac %.3f'%(c.get('us_per_step',0), c.get('frac',0)), 'cpu', (d.get('cpu_baseline') or {}).get('value'), d.get('window_phase'))
"
}

exp_cpc2() {
# C3 GEMM chunk size around 2 per CU with the unsplit small levels
O=gpurun_out/r03cpc2
mkdir -p $O
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 600 python scripts/exp_time.py --steps 512 --short-reps 8 --rounds 3 --windows 20 --window-reps 9 --variants ";GLE_CG_PER_CU=1.5;GLE_CG_PER_CU=3" --tag cpc2 > $O/cpc2.jsonl 2> $O/cpc2.err || { echo "cpc2 failed"; tail -20 $O/cpc2.err; exit 1; }
python3 -c "
import json, statistics as st
for l in open('$O/cpc2.jsonl'):
    d=json.loads(l); r=d['short_reps_ms']
    print('%-20s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'reps mean %.4f'%st.mean(r), 'w20 %.4f'%(d['window_ms']['20']/20), d['finite'])
"
}

exp_c5alone() {
# C5: the chain with and without the far field (GLE_DBG_NO_LADDER=1: no ladder levels, wrong
# numbers, timing only), chain launches device-stamped: how much the K-hat stream costs the chain.
O=gpurun_out/r03c5alone
mkdir -p $O
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 600 python -u scripts/exp_time.py --config C5 --ntraj 32 --steps 256 --short 20 --rounds 2 --chainprof 1 --variants ";GLE_DBG_NO_LADDER=1" --tag c5alone > $O/c5alone.jsonl 2> $O/c5alone.err || { echo "c5alone failed"; tail -20 $O/c5alone.err; exit 1; }
python3 -c "
import json
for l in open('$O/c5alone.jsonl'):
    d=json.loads(l)
    print('%-22s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'chain us/step', d.get('chain_us_per_step'))
"
}

exp_c5skip() {
# C5 step decomposition (timing only, wrong numbers): no far-field GEMMs (GLE_DBG_SKIP=1), no
# transforms (6), neither (7), against the plan; chain launches device-stamped.
O=gpurun_out/r03c5skip
mkdir -p $O
SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 600 python -u scripts/exp_time.py --config C5 --ntraj 32 --steps 256 --short 20 --rounds 2 --chainprof 1 --variants ";GLE_DBG_SKIP=1;GLE_DBG_SKIP=6;GLE_DBG_SKIP=7" --tag c5skip > $O/c5skip.jsonl 2> $O/c5skip.err || { echo "c5skip failed"; tail -20 $O/c5skip.err; exit 1; }
python3 -c "
import json
for l in open('$O/c5skip.jsonl'):
    d=json.loads(l)
    print('%-22s'%d['variant'], 'long %.4f'%d['ms_per_step'], 'chain us/step', d.get('chain_us_per_step'))
"
}

[ $# -gt 0 ] || { echo "experiments: c5skip c5alone cpc2 final4 split fftp lines c3cpc kc ab1 audit batch c2p c2w c5b c5cpc c5exp c5f c5s evidence fpot interf nw ph win2 xq"; exit 2; }
for e in "$@"; do "exp_$e" || exit 1; done
