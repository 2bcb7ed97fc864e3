cd $GRAFT_REPO_ROOT
for scn in mixed polygon line; do
  for v in base nolsa; do
    ABL_SCN=$scn ABL_N=24 ABL_B=8192 GSM_LIB_PATH=gs-marl_amd/gsmarl_amd/lib/ablate/$v.so timeout -k 10 120 python tools/ablate.py || exit 1
  done
done
