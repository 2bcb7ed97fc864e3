# Round-5 call: the headline prologue reorder (state loads before the pace
# arrival and the zeroing stores): rollout tests, A/B against HEAD's build,
# launch-timeline stamps of the new build.
cd $GRAFT_REPO_ROOT; O=gpurun_out/cd; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_roll.py tests/test_gpu_roll_ragged.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_roll.log 2>&1 || { tail -30 $O/pytest_roll.log; exit 3; }
tail -1 $O/pytest_roll.log
AB_LINES="driver h" bash tools/gpu.sh ab dab head || exit 5
S=$GRAFT_REPO_ROOT/gs-marl_amd/gsmarl_amd/lib/ablate/stamps.so
GSM_LIB_PATH=$S STAMPS_NPZ=$O/h20.npz timeout -k 10 200 python3 tools/stamps_h_timeline.py > $O/h20.json 2> $O/h20.err || exit 1
python3 tools/stamps_h_spread.py $O/h20.npz > $O/h20_spread.json
