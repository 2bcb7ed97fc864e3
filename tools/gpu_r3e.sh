set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r3_e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_roll.py tests/test_gpu_rollout.py tests/test_gpu_oracle_direct.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_roll.log 2>&1 || { tail -40 $O/pytest_roll.log; exit 2; }
tail -1 $O/pytest_roll.log
bash tools/gpu_ab.sh r3_e_ab graph lag2
