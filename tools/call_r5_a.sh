# Round-5 A/B call: rollout tests (product and checked builds), then the
# library against HEAD's build (ablate/head.so) on driver / h / c2 / c4, the C4
# placement knob, and PMC traffic of C4 and C2.
cd $GRAFT_REPO_ROOT; O=gpurun_out/ca; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_roll_ragged.py tests/test_gpu_roll.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_roll.log 2>&1 || { tail -30 $O/pytest_roll.log; exit 3; }
tail -1 $O/pytest_roll.log
GSM_LIB_PATH=$GRAFT_REPO_ROOT/gs-marl_amd/gsmarl_amd/lib/ablate/checked.so timeout -k 10 500 python -u -m pytest tests/test_gpu_roll_ragged.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_checked.log 2>&1 || { tail -30 $O/pytest_checked.log; exit 3; }
tail -1 $O/pytest_checked.log
AB_LINES="driver h c4 c2" bash tools/gpu.sh ab cab head || exit 5
bash tools/gpu.sh envsweep cx c4 GSM_PLACE_XCD 0 1 || exit 2
PMC_CONFIG=c4 PMC_SET="traffic" bash tools/pmc_quick.sh pq_c4 libgsm.so ablate/head.so || exit 4
GSM_PLACE_XCD=0 PMC_CONFIG=c4 PMC_SET="traffic" bash tools/pmc_quick.sh pq_c4x0 libgsm.so || exit 4
PMC_CONFIG=c2 PMC_SET="traffic" bash tools/pmc_quick.sh pq_c2 libgsm.so ablate/head.so || exit 4
