# Round-5 call: the eager env.step at H — host issue vs device time, two
# launches vs the one-launch form (the rollout kernel with K = 1 on the
# round-5 one-hop prefix), and a rocprof kernel summary of each.
cd $GRAFT_REPO_ROOT; O=gpurun_out/cg; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python -u tools/probe_eager.py > $O/probe_two.json 2> $O/probe_two.err || { tail -20 $O/probe_two.err; exit 3; }
cat $O/probe_two.json
GSM_EAGER_ONE_LAUNCH=1 timeout -k 10 200 python -u tools/probe_eager.py > $O/probe_one.json 2> $O/probe_one.err || { tail -20 $O/probe_one.err; exit 4; }
cat $O/probe_one.json
timeout -k 10 200 python -u bench.py --eager --steps 200 --warmup 20 > $O/bench_two.json 2> $O/bench_two.err || exit 5
GSM_EAGER_ONE_LAUNCH=1 timeout -k 10 200 python -u bench.py --eager --steps 200 --warmup 20 > $O/bench_one.json 2> $O/bench_one.err || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_two -o run -- python3 tools/probe_eager.py --steps 300 > $O/prof_two.log 2>&1 || exit 7
GSM_EAGER_ONE_LAUNCH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_one -o run -- python3 tools/probe_eager.py --steps 300 > $O/prof_one.log 2>&1 || exit 8
grep -h '"ms_per_step"' $O/bench_two.json $O/bench_one.json | python3 -c 'import sys,json; [print(json.loads(l)["ms_per_step"]) for l in sys.stdin]'
