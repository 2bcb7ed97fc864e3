# Round-5 call: the headline rollout's final state stored before its tail
# emissions, and the eager kernels' loads at priority 3: rollout + parity
# tests, then a same-box A/B (h, driver, eager lines) against the previous
# commit's build, and the eager probe of both launch forms.
cd $GRAFT_REPO_ROOT; O=gpurun_out/cj; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_roll.py tests/test_gpu_rollout.py tests/test_gpu_oracle_direct.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
AB_LINES="h driver eager" bash tools/gpu.sh ab cj prev || exit 5
for v in lib prev; do
  L=""; [ $v = lib ] || L=gs-marl_amd/gsmarl_amd/lib/ablate/$v.so
  GSM_LIB_PATH=$L GSM_EAGER_ONE_LAUNCH=1 timeout -k 10 200 python -u tools/probe_eager.py > $O/probe_one_$v.json 2> $O/probe_one_$v.err || exit 7
  cat $O/probe_one_$v.json
done
