set -o pipefail
O=gpurun_out/r06/mp; mkdir -p $O
for r in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/p1x64_$r.json 2> $O/p1x64_$r.err && \
timeout -k 10 300 python bench.py --gpus 2 --same-device --dist-backend gloo --ntraj 32 --steps 20 --warmup 5 --no-cpu-baseline > $O/p2x32_$r.json 2> $O/p2x32_$r.err && \
timeout -k 10 300 python bench.py --gpus 4 --same-device --dist-backend gloo --ntraj 16 --steps 20 --warmup 5 --no-cpu-baseline > $O/p4x16_$r.json 2> $O/p4x16_$r.err || exit 1
done
for f in $O/*.json; do python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1].split('/')[-1], round(d['value']), round(d['ms_per_step']*1e3,2), d['config']['ntraj_total'], d['window_phase']['scan_ms_per_step'])" $f; done
