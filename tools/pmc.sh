# rocprofv3 PMC passes over a short eager bench run (one counter group per pass).
# Usage: bash tools/pmc.sh TAG [extra bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-pmc}; shift
OUT="$GRAFT_REPO_ROOT/gpurun_out/${TAG}"
mkdir -p "$OUT"
cd /tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
# PMC_GRAPH=1: graph replay (lagged-emission step kernels) instead of eager launches
# PMC_ROLL=1: one fused rollout graph of 100 steps (no warmup / alignment graphs)
LAUNCH="--eager --warmup 10"; [ -n "$PMC_GRAPH" ] && LAUNCH="--no-roll --warmup 10"
[ -n "$PMC_ROLL" ] && LAUNCH="--warmup 0 --no-align"
BENCH="$GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-kernel-timing --settle-ms 0 $LAUNCH --steps 100 $*"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python $BENCH > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; }
done
python "$GRAFT_REPO_ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
