# Timing only (no PMC) of ablation builds: bash tools/abl_time.sh NAME...  (ABL_N/ABL_B/ABL_SCN pick the config)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for name in "$@"; do
  GSM_LIB_PATH=gs-marl_amd/gsmarl_amd/lib/ablate/$name.so timeout -k 10 120 python tools/ablate.py 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('$name', {k: round(v*1e3,2) for k,v in d.items() if k.endswith('_ms')})" || exit 1
done
