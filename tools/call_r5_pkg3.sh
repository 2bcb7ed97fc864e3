# Round-5 final package, part 3: the GPU suite + smoke, every bench line, and
# rocprof kernel summaries, on the code object the PMC was collected on.
cd $GRAFT_REPO_ROOT
bash tools/gpu.sh tests r5f || exit 2
bash tools/gpu.sh lines r5f || exit 4
bash tools/gpu.sh prof r5f h c4 eager policyg buffer driver c2 c3 || exit 6
# the checked build (every granule / slab address tested against its
# allocation) over the rollout tests, once, on these sources
GSM_LIB_PATH=$GRAFT_REPO_ROOT/gs-marl_amd/gsmarl_amd/lib/ablate/checked.so timeout -k 10 600 python -u -m pytest tests/test_gpu_roll.py tests/test_gpu_roll_ragged.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5f/pytest_checked.log 2>&1 || { tail -30 gpurun_out/r5f/pytest_checked.log; exit 7; }
tail -1 gpurun_out/r5f/pytest_checked.log
