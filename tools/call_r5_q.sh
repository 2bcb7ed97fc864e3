# Round-5 call: why the h line's timed 100-step graphs run ~760-800 us while
# the roofline's settled ones run ~680 (same env, same process): per-chunk
# HIP events in the timed region (GSM_BENCH_CHUNK_US) with the timed graph
# in slot 0 (default), in the settle loop's slot 3, and slot 0 re-captured
# right before the region.
cd $GRAFT_REPO_ROOT; O=gpurun_out/cu; mkdir -p $O
for r in 1 2; do
  for v in s0 s3 rc; do
    case $v in s0) e="";; s3) e="GSM_BENCH_TIMED_SLOT=3";; rc) e="GSM_BENCH_RECAPTURE=1";; esac
    env $e GSM_BENCH_CHUNK_US=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/h_${v}_$r.json 2> $O/h_${v}_$r.err || exit 3
    echo "$v: $(grep 'timed region chunks' $O/h_${v}_$r.err) line $(python3 -c "import json; print(json.load(open('$O/h_${v}_$r.json'))['ms_per_step'])")"
  done
done
