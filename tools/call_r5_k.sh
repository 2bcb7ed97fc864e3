# Round-5 call: the eager step per config, two launches vs one launch
# (tools/probe_eager.py device time per step).
cd $GRAFT_REPO_ROOT; O=gpurun_out/ck; mkdir -p $O
for c in "24 8192" "3 4096" "96 1024" "12 8192" "6 8192"; do
  set -- $c
  for one in 0 1; do
    GSM_EAGER_ONE_LAUNCH=$one timeout -k 10 200 python -u tools/probe_eager.py --agents $1 --envs $2 --steps 1000 >> $O/probe.jsonl 2>> $O/probe.err || { tail -20 $O/probe.err; exit 3; }
  done
done
cat $O/probe.jsonl
