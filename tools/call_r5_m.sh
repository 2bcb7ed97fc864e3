# Round-5 call: per-wave pacing in the ragged (C4) rollout: the ragged GPU
# tests, then a same-box A/B of the c4 line against the previous build.
cd $GRAFT_REPO_ROOT; O=gpurun_out/co; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_roll_ragged.py tests/test_gpu_ragged.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
AB_LINES="c4" bash tools/gpu.sh ab co prev || exit 5
