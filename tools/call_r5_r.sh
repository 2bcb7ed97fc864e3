# Round-5 call: the h line's timed 100-step graphs (~750-800 us) against the
# same graphs settled (~680): per-chunk events under variants of what runs
# before the region — default, no collector pass, no warmup graph, a longer
# settle loop.
cd $GRAFT_REPO_ROOT; O=gpurun_out/cv; mkdir -p $O
for r in 1 2; do
  for v in def nogc now settle200; do
    e=""; a=""
    case $v in nogc) e="GSM_BENCH_NO_GC=1";; now) a="--warmup 0";; settle200) a="--settle-ms 200";; esac
    env $e GSM_BENCH_CHUNK_US=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline $a > $O/h_${v}_$r.json 2> $O/h_${v}_$r.err || exit 3
    echo "$v: $(grep 'timed region chunks' $O/h_${v}_$r.err) line $(python3 -c "import json; d=json.load(open('$O/h_${v}_$r.json')); print(d['ms_per_step'], d['roofline']['mean_launch_us'])")"
  done
done
