# Round-5 call: the packed C2 rollout at 2 envs per wave (library) against 4
# (HEAD's build) and 1 (ablate/pack1.so): rollout tests at C2 shapes and the
# new C4 placement test, then A/B of the C2 line.
cd $GRAFT_REPO_ROOT; O=gpurun_out/ce; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_roll.py tests/test_gpu_rollout.py tests/test_gpu_oracle_direct.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_c2.log 2>&1 || { tail -30 $O/pytest_c2.log; exit 3; }
tail -1 $O/pytest_c2.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_roll_ragged.py -m gpu -x -q -k xcd --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_xcd.log 2>&1 || { tail -30 $O/pytest_xcd.log; exit 3; }
tail -1 $O/pytest_xcd.log
AB_LINES="c2" bash tools/gpu.sh ab eab head pack1 || exit 5
