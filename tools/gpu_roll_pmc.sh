# PMC instruction counts (one pass) of the rollout kernel for the library and
# ablation builds: bash tools/gpu_roll_pmc.sh TAG [names...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
for name in default "$@"; do
  lib=""; [ "$name" != default ] && lib=gs-marl_amd/gsmarl_amd/lib/ablate/$name.so
  GSM_LIB_PATH=$lib timeout -k 10 120 python tools/probe_roll.py 2>/dev/null | sed "s/^/$name /" || exit 5
  ( cd /tmp && GSM_LIB_PATH=${lib:+$GRAFT_REPO_ROOT/$lib} timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$GRAFT_REPO_ROOT/$O/$name/p1" -o run -- python "$GRAFT_REPO_ROOT/tools/probe_roll.py" --reps 2 > "$GRAFT_REPO_ROOT/$O/$name.log" 2>&1 ) || exit 6
  python tools/pmc_summary.py $O/$name | python -c "
import json,sys; d=json.load(sys.stdin); r=d.get('roll',{}).get('derived',{}); print('$name', {k: round(v/100,1) for k,v in r.items() if 'per_wave' in k})"
done
