#!/bin/bash
# GPU-box evidence runs, one entry point (replaces the per-round gpu_r0*_*.sh launchers).
#
#   scripts/gpu_evidence.sh <outdir> <task> [<task> ...]
#
# tasks (each step bounded by its own timeout; the script stops at the first failure):
#   tests      the -m gpu parity suite (one pytest process)
#   lines      bench lines: C3 driver 20/5, C3 512 steps, C2 1 trajectory
#   c5         C5 32-trajectory line over one period of the largest level (256 steps)
#   rccl       C3 20/5 and 512-step lines plain vs world-1 torchrun/nccl (stepper first, and RCCL
#              first via --early-collective), interleaved twice; 8-rank same-device gloo rehearsal
#   trace      rocprofv3 kernel trace + stats of the C3 bench, summarised
#   pmc        FETCH_SIZE / WRITE_SIZE passes over the C3 bench (cgemm and chain traffic)
#   trace_c5 / pmc_c5   the same for the C5 line; trace_c2 the C2 line's trace
#   blocklen   bench lines at several first block lengths (BLS, CONFIGS, ROUNDS)
#   c5run      md.Run wall time per run at C5 (scripts/c5_run_timing.py: noise, stepping, MD{j}.nc)
#   c1         the C1 host-driver step (scripts/c1_driver_timing.py)
#   c4shape    BASELINE config 4's shape (8 ranks x 64 trajectories) as 8 gloo ranks on one GPU
#   noiseshare per-rank host factorisation of the C5 noise split over a node's 8 ranks (no GPU)
#   rehearse_share  8 same-device gloo ranks with streamed C3 noise: per-rank setup / factorisations
#   negf       GLE ensemble current vs the NEGF Landauer current (tests/test_gpu_negf.py)
#   ab         experiment libraries x GLE_* variants, interleaved (LIBS, VARIANTS, ROUNDS, EXPARGS,
#              TIMELINES=1 for per-workgroup chain timelines); build them with make experiments
#              EXPNAME=.. EXPFLAGS=.. or scripts/build_variant.sh <name> <git-rev>
#   runtime / queues   the HIP runtime and hardware-queue studies of round 5 (profiles/r05)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:?outdir}
shift
mkdir -p $O
fail() { echo "FAILED: $1"; [ -f "$2" ] && tail -30 "$2"; exit 1; }
summ() {
python3 - "$@" <<'PY'
import json, sys
for p in sys.argv[1:]:
    try:
        d = json.loads([l for l in open(p) if l.startswith("{")][-1])
    except Exception as e:
        print(p, "unreadable", e); continue
    r = d.get("roofline", {}); c = d.get("chain_roofline", {})
    print("%-28s %10.0f traj-steps/s %6.1f us/step  roof %.3f  chain %.1f us/step frac %.3f  n_gpus %s  phase %s" % (
        p.split("/")[-1], d["value"], d["ms_per_step"] * 1e3, r.get("frac", 0), c.get("us_per_step", 0), c.get("frac", 0),
        d["n_gpus"], (d.get("window_phase") or {}).get("scan_ms_per_step")))
PY
}
TR="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node"
port=29611
for task in "$@"; do
case $task in
tests)
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
    || fail tests $O/gpu_tests.log
  tail -2 $O/gpu_tests.log ;;
lines)
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3_20x5.json 2> $O/bench_c3_20x5.err || fail b20 $O/bench_c3_20x5.err
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || fail b512 $O/bench_c3.err
  timeout -k 10 300 python bench.py --config C2 --ntraj 1 --steps 256 --warmup 32 > $O/bench_c2.json 2> $O/bench_c2.err || fail c2 $O/bench_c2.err
  summ $O/bench_c3_20x5.json $O/bench_c3.json $O/bench_c2.json ;;
c1)
  timeout -k 10 300 python scripts/c1_driver_timing.py --nmd 1024 > $O/c1_driver_timing.json 2> $O/c1_driver_timing.err || fail c1 $O/c1_driver_timing.err
  cat $O/c1_driver_timing.json ;;
noiseshare)
  # host only: per-rank factorisation time of the C5 noise spectra when 8 ranks of a node split them
  timeout -k 10 600 python scripts/noise_share_timing.py --world 8 --workers 16 > $O/noise_share_c5.json 2> $O/noise_share_c5.err || fail noiseshare $O/noise_share_c5.err
  cat $O/noise_share_c5.json ;;
rehearse_share)
  # 8 ranks on one GPU over gloo with the C3 noise streamed: every rank's setup, noise phase and
  # factorisation count (noise.NodeShare: the counts add up to one rank's)
  timeout -k 10 600 python bench.py --gpus 8 --same-device --dist-backend gloo --ntraj 8 --stream-noise --steps 8 --warmup 2 \
    --fill 16 --no-cpu-baseline > $O/rehearsal_share8.json 2> $O/rehearsal_share8.err || fail share8 $O/rehearsal_share8.err
  timeout -k 10 600 python bench.py --ntraj 8 --stream-noise --steps 8 --warmup 2 --fill 16 --no-cpu-baseline \
    > $O/rehearsal_share1.json 2> $O/rehearsal_share1.err || fail share1 $O/rehearsal_share1.err
  python3 -c "import json,sys
for f in sys.argv[1:]:
    d=json.loads([l for l in open(f) if l.startswith('{')][-1]); print(f.split('/')[-1], d['n_gpus'], d['setup_ranks'])" $O/rehearsal_share8.json $O/rehearsal_share1.json ;;
c4shape)
  # BASELINE config 4's shape (512 trajectories over 8 ranks, 64 each) rehearsed on one GPU: 8 gloo
  # ranks on device 0 (the control flow, the node-shared noise factorisation and the reduce; the
  # rate is 8 ranks time-sharing one GPU, not the 8-GPU node's)
  timeout -k 10 900 python bench.py --gpus 8 --same-device --dist-backend gloo --ntraj 64 --steps 20 --warmup 5 \
    --no-cpu-baseline > $O/c4shape_8x64.json 2> $O/c4shape_8x64.err || fail c4shape $O/c4shape_8x64.err
  summ $O/c4shape_8x64.json ;;
c5run)
  timeout -k 10 900 python scripts/c5_run_timing.py --runs ${RUNS:-3} > $O/c5_run_timing.json 2> $O/c5_run_timing.log || fail c5run $O/c5_run_timing.log
  cat $O/c5_run_timing.json ;;
negf)
  timeout -k 10 300 python -u -m pytest tests/test_gpu_negf.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/negf.log 2>&1 || fail negf $O/negf.log
  tail -3 $O/negf.log ;;
c5)
  timeout -k 10 600 python bench.py --config C5 --ntraj 32 --steps 256 --warmup 32 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || fail c5 $O/bench_c5.err
  summ $O/bench_c5.json ;;
rccl)
  python3 -c "import torch; print('stream priority range (least, greatest):', torch.cuda.Stream.priority_range())"
  for r in 1 2; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/rccl_plain20_$r.json 2> $O/rccl_plain20_$r.err || fail plain $O/rccl_plain20_$r.err
    port=$((port+1))
    timeout -k 10 300 $TR 1 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/rccl_nccl20_$r.json 2> $O/rccl_nccl20_$r.err || fail nccl $O/rccl_nccl20_$r.err
    port=$((port+1))
    timeout -k 10 300 $TR 1 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --early-collective > $O/rccl_ncclfirst20_$r.json 2> $O/rccl_ncclfirst20_$r.err || fail ncclfirst $O/rccl_ncclfirst20_$r.err
    timeout -k 10 300 python bench.py --no-cpu-baseline > $O/rccl_plain512_$r.json 2> $O/rccl_plain512_$r.err || fail plain512 $O/rccl_plain512_$r.err
    port=$((port+1))
    timeout -k 10 300 $TR 1 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 1 --no-cpu-baseline > $O/rccl_nccl512_$r.json 2> $O/rccl_nccl512_$r.err || fail nccl512 $O/rccl_nccl512_$r.err
  done
  timeout -k 10 400 python bench.py --gpus 8 --same-device --dist-backend gloo --ntraj 8 --noise white --steps 20 --warmup 5 \
    --no-cpu-baseline > $O/rehearsal_gloo8.json 2> $O/rehearsal_gloo8.err || fail gloo8 $O/rehearsal_gloo8.err
  summ $O/rccl_*.json $O/rehearsal_gloo8.json ;;
runtime)
  # which HIP runtime the stepper runs on: plain (the library's /opt/rocm), torch imported first (torch's
  # bundled copy), torchrun world-1 over gloo (torch first, no RCCL) and over nccl; interleaved twice
  for r in 1 2; do for K in 20 512; do
    W=$([ $K = 20 ] && echo 5 || echo 64)
    timeout -k 10 300 python bench.py --steps $K --warmup $W --no-cpu-baseline > $O/rt_plain$K\_$r.json 2> $O/rt_plain$K\_$r.err || fail plain $O/rt_plain$K\_$r.err
    timeout -k 10 300 python -c "import torch, runpy, sys; sys.argv = ['bench.py', '--steps', '$K', '--warmup', '$W', '--no-cpu-baseline']; runpy.run_path('bench.py', run_name='__main__')" > $O/rt_torchfirst$K\_$r.json 2> $O/rt_torchfirst$K\_$r.err || fail torchfirst $O/rt_torchfirst$K\_$r.err
    port=$((port+1))
    timeout -k 10 300 $TR 1 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 1 --dist-backend gloo --steps $K --warmup $W --no-cpu-baseline > $O/rt_gloo$K\_$r.json 2> $O/rt_gloo$K\_$r.err || fail gloo $O/rt_gloo$K\_$r.err
    port=$((port+1))
    timeout -k 10 300 $TR 1 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 1 --steps $K --warmup $W --no-cpu-baseline > $O/rt_nccl$K\_$r.json 2> $O/rt_nccl$K\_$r.err || fail nccl $O/rt_nccl$K\_$r.err
  done; done
  summ $O/rt_*.json
  python3 -c "
import json, glob
for p in sorted(glob.glob('$O/rt_*_1.json')):
    d = json.loads([l for l in open(p) if l.startswith('{')][-1]); print(p.split('/')[-1], d.get('runtime_libs'))" ;;
ab)
  # experiment libraries (LIBS, e.g. "base cur": scripts/build_variant.sh / make experiments) x
  # GLE_* VARIANTS, one process per (lib, variant), ROUNDS interleaved; then chain timelines per lib
  : > $O/ab.jsonl
  for r in $(seq 1 ${ROUNDS:-3}); do for lib in ${LIBS:?}; do
    SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_$lib.so timeout -k 10 300 python scripts/exp_time.py --tag $lib \
      --variants "${VARIANTS:-}" --short-reps 16 ${EXPARGS:-} >> $O/ab.jsonl 2>> $O/ab.err || fail "ab $lib" $O/ab.err
  done; done
  python3 - $O/ab.jsonl <<'PY'
import json, sys, collections
import numpy as np
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        agg[(d["tag"], d["variant"])].append((d["ms_per_step"] * 1e3, np.median(d["short_reps_ms"]) * 1e3,
                                              d.get("cgemm_tflops", 0.0), d.get("cgemm_avg_us", 0.0)))
for k, v in agg.items():
    print("%-8s %-36s 512-step %s | 20-step median %s%s" % (k[0], k[1] or "(default)", " ".join("%.2f" % x[0] for x in v),
          " ".join("%.2f" % x[1] for x in v),
          (" | cgemm TF/s %s avg us %s" % (" ".join("%.1f" % x[2] for x in v), " ".join("%.1f" % x[3] for x in v)))
          if v[0][2] else ""))
PY
  if [ -n "$TIMELINES" ]; then for lib in $LIBS; do for v in "GLE_DBG_NO_LADDER=1" "GLE_PIECE_SLACK=0"; do
    env $v GLE_CHAIN_DBG=700 SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_$lib.so timeout -k 10 200 python scripts/exp_time.py \
      --tag "$lib $v" --steps 256 > $O/tl.$lib.$v.json 2> $O/tl.$lib.$v.err || fail "tl $lib" $O/tl.$lib.$v.err
    echo "== $lib $v"; grep "chain dbg" $O/tl.$lib.$v.err
  done; done; fi ;;
queues)
  # hardware-queue placement of the stepper's streams (experiment build, GLE_QUEUE_MODE) against a
  # world-1 nccl group joined before / after the stepper, one process per (mode, order), 2 rounds
  : > $O/queues.jsonl
  for r in 1 2; do for q in ${QMODES:-0 1 2}; do for d in none before after; do
    port=$((port+1))
    GLE_QUEUE_MODE=$q SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so timeout -k 10 300 python scripts/exp_time.py \
      --tag q$q-$d --dist $d --port $port --short-reps 16 >> $O/queues.jsonl 2>> $O/queues.err || fail "queues $q $d" $O/queues.err
  done; done; done
  python3 - $O/queues.jsonl <<'PY'
import json, sys, collections
import numpy as np
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if not l.startswith("{"):
        continue  # RCCL's version banner
    d = json.loads(l)
    agg[d["tag"]].append((d["ms_per_step"] * 1e3, np.median(d["short_reps_ms"]) * 1e3))
for k, v in agg.items():
    print("%-12s 512-step %s   20-step median %s" % (k, " ".join("%.2f" % x[0] for x in v), " ".join("%.2f" % x[1] for x in v)))
PY
  ;;
trace|trace_c5|trace_c2)
  K=cgemm
  case $task in
    trace) A="--no-cpu-baseline"; n=c3 ;;
    trace_c5) A="--config C5 --ntraj 32 --steps 256 --warmup 32 --no-cpu-baseline"; n=c5 ;;
    trace_c2) A="--config C2 --ntraj 1 --steps 256 --warmup 32 --no-cpu-baseline"; n=c2; K=contract ;;
  esac
  mkdir -p $O/prof_$n
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$n -o run -- \
    python3 bench.py $A > $O/prof_$n/bench.json 2> $O/prof_$n/bench.err || fail trace $O/prof_$n/bench.err
  N=$(python3 -c "import json;print(json.load(open('$O/prof_$n/bench.json'))['roofline']['launches'])")
  python3 scripts/trace_summary.py $O/prof_$n/run_kernel_trace.csv --steps --gaps --last $K $N --skip $N > $O/prof_$n/summary.txt
  tail -8 $O/prof_$n/summary.txt ;;
blocklen)
  # bench lines at first block lengths BLS (0: the planner's choice), CONFIGS among c3 c2 c5, ROUNDS interleaved
  for r in $(seq 1 ${ROUNDS:-2}); do for c in ${CONFIGS:-c3 c2}; do for bl in ${BLS:-0 4}; do
    case $c in
      c3) A="" ;; c2) A="--config C2 --ntraj 1 --steps 256 --warmup 32" ;; c5) A="--config C5 --ntraj 32 --steps 256 --warmup 32" ;;
    esac
    timeout -k 10 400 python bench.py --no-cpu-baseline --block-len $bl $A > $O/${c}_bl${bl}_$r.json 2> $O/${c}_bl${bl}_$r.err \
      || fail "blocklen $c $bl" $O/${c}_bl${bl}_$r.err
  done; done; done
  summ $O/*_bl*_*.json ;;
pmc|pmc_c5)
  if [ $task = pmc ]; then A="--no-cpu-baseline"; n=c3; cfg="--config C3 --ntraj 64"; else A="--config C5 --ntraj 32 --steps 256 --warmup 32 --no-cpu-baseline"; n=c5; cfg="--config C5 --ntraj 32"; fi
  mkdir -p $O/pmc_$n
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 600 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$n/$c -o run -- \
      python3 bench.py $A > $O/pmc_$n/$c.json 2> $O/pmc_$n/$c.err || fail "pmc $c" $O/pmc_$n/$c.err
  done
  python3 scripts/pmc_summary.py $O/pmc_$n $O/pmc_$n/traffic_cgemm.json --kernel cgemm_kernel $cfg
  python3 scripts/pmc_summary.py $O/pmc_$n $O/pmc_$n/traffic_chain.json --kernel chain_kernel $cfg --last ${CHAIN_LAST:-512} --skip-chain-window 0 ;;
*)
  echo "unknown task $task"; exit 2 ;;
esac
done
