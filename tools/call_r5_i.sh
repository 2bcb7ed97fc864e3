# Round-5 call: the eager step and emit kernels with their loads issued at
# priority 3 (then 1): parity tests of the eager path, then a same-box A/B
# of the eager line against HEAD's build, and the eager probe (two launches,
# and the one-launch form with the rollout's start priorities).
cd $GRAFT_REPO_ROOT; O=gpurun_out/ci; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_roll.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
AB_LINES="eager" bash tools/gpu.sh ab ci head || exit 5
timeout -k 10 200 python -u tools/probe_eager.py > $O/probe_two.json 2> $O/probe_two.err || exit 6
GSM_EAGER_ONE_LAUNCH=1 timeout -k 10 200 python -u tools/probe_eager.py > $O/probe_one.json 2> $O/probe_one.err || exit 7
cat $O/probe_two.json $O/probe_one.json
