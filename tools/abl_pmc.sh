# Time + VALU/SALU counts (one SQ PMC pass) of ablation builds made by
# tools/ablate.sh build. Usage (GPU box): bash tools/abl_pmc.sh TAG NAME...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
O="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$O"
for name in "$@"; do
  lib="$GRAFT_REPO_ROOT/gs-marl_amd/gsmarl_amd/lib/ablate/$name.so"
  GSM_LIB_PATH=$lib timeout -k 10 120 python tools/ablate.py > "$O/$name.time.json" 2> "$O/$name.time.err" || { tail -5 "$O/$name.time.err"; exit 1; }
  cat "$O/$name.time.json"
  cd /tmp
  GSM_LIB_PATH=$lib timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR --output-format csv -d "$O/$name/p1" -o run -- python "$GRAFT_REPO_ROOT/tools/ablate.py" > "$O/$name.pmc.log" 2>&1 || { tail -5 "$O/$name.pmc.log"; exit 2; }
  cd "$GRAFT_REPO_ROOT"
  python tools/pmc_summary.py "$O/$name" > "$O/$name/summary.txt" 2>&1
  python - "$O/$name/summary.txt" <<'PY'
import json, sys
t = open(sys.argv[1]).read(); d = json.loads(t[t.index("{"):])
for k, v in d.items():
    print(" ", k, {a: round(b, 1) for a, b in v["derived"].items() if "per_wave" in a})
PY
done
