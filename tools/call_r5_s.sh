# Round-5 call: bench.py with the collector pass and the alignment's capture
# moved before the settle loop (nothing idles the GPU between the settle loop
# and the timed region; eager / closed-loop lines settle too): the driver
# command three times, then the other lines once (chunk events on h).
cd $GRAFT_REPO_ROOT; O=gpurun_out/cw; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$r.json 2> $O/driver_$r.err || { tail -20 $O/driver_$r.err; exit 3; }
  python3 -c "import json; d=json.load(open('$O/driver_$r.json')); print('driver', d['ms_per_step'], d['timed_region'])"
done
GSM_BENCH_CHUNK_US=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/h.json 2> $O/h.err || exit 4
grep 'timed region chunks' $O/h.err
for l in h driver c2 c3 c4 eager policy policyg buffer n6 n12; do bash tools/gpu.sh lines cw $l || exit 5; done
