# Round-5 call: start priorities for the headline rollout's first two
# iterations (entry 3, step 0 at 2, step 1 at 1; gsm_device.h start_prio):
# rollout tests, the launch timeline of the stamps build, then a same-box A/B
# against HEAD's build on the h and driver lines.
cd $GRAFT_REPO_ROOT; O=gpurun_out/chh; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_roll.py tests/test_gpu_rollout.py tests/test_gpu_oracle_direct.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
STAMPS_NPZ=$O/k20.npz GSM_LIB_PATH=$PWD/gs-marl_amd/gsmarl_amd/lib/ablate/stamps.so timeout -k 10 300 python -u tools/stamps_h_timeline.py > $O/timeline.txt 2>&1 || { tail -20 $O/timeline.txt; exit 4; }
AB_LINES="h driver" bash tools/gpu.sh ab chh head || exit 5
