# Round-5 call: start priorities in the tile (C3) rollout: tile rollout tests,
# then a same-box A/B of the c3 line against the previous build.
cd $GRAFT_REPO_ROOT; O=gpurun_out/cp; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_roll.py tests/test_gpu_rollout.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
AB_LINES="c3" bash tools/gpu.sh ab cp prev || exit 5
