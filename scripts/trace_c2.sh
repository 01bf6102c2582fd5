# rocprofv3 kernel trace + stats of the C2 (1 trajectory) bench line, summarised like the C3 / C5 traces
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?outdir}/prof_c2; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- \
  python3 bench.py --config C2 --ntraj 1 --steps 256 --warmup 32 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
N=$(python3 -c "import json;print(json.load(open('$O/bench.json'))['roofline']['launches'])")
python3 scripts/trace_summary.py $O/run_kernel_trace.csv --steps --gaps --last contract $N --skip $N > $O/summary.txt
tail -30 $O/summary.txt
