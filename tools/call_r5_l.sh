# Round-5 call: the one-launch eager step as the default at 6-24 agents
# (decided at gsm_bind): the whole GPU suite, the eager line, and the eager
# probe of both forms at H.
cd $GRAFT_REPO_ROOT; O=gpurun_out/cm; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --eager --steps 200 --warmup 20 --no-cpu-baseline > $O/eager_$r.json 2> $O/eager_$r.err || exit 4
  GSM_EAGER_ONE_LAUNCH=0 timeout -k 10 200 python3 bench.py --eager --steps 200 --warmup 20 --no-cpu-baseline > $O/eager_two_$r.json 2> $O/eager_two_$r.err || exit 5
done
grep -h ms_per_step $O/eager_*.json | python3 -c 'import sys,json; [print(json.loads(l)["ms_per_step"]) for l in sys.stdin]'
