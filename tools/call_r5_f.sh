# Round-5 call: the headline sweep with transposed-bit rows (plain VALU) in the
# fused rollout: rollout tests (rollout vs the ballot-form step kernels, oracle),
# then A/B against HEAD's build on h / driver.
cd $GRAFT_REPO_ROOT; O=gpurun_out/cf; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_roll.py tests/test_gpu_rollout.py tests/test_gpu_oracle_direct.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
AB_LINES="h driver" bash tools/gpu.sh ab fab2 head || exit 5
