# Fused rollout on the GPU: its tests, probe_roll for the library and any
# ablation builds named, then PMC passes over probe_roll.
# Usage: bash tools/gpu_roll.sh TAG [ablation names...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-roll}; shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_roll.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -3 $O/pytest.log
timeout -k 10 120 python tools/probe_roll.py > $O/probe.json 2>/dev/null || exit 4
cat $O/probe.json
for name in "$@"; do
  GSM_LIB_PATH=gs-marl_amd/gsmarl_amd/lib/ablate/$name.so timeout -k 10 120 python tools/probe_roll.py 2>/dev/null | sed "s/^/$name /" || exit 5
done
if [ -n "$ROLL_PMC" ]; then
  cd /tmp
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d "$GRAFT_REPO_ROOT/$O/p$i" -o run -- python "$GRAFT_REPO_ROOT/tools/probe_roll.py" --reps 3 > "$GRAFT_REPO_ROOT/$O/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$GRAFT_REPO_ROOT/$O/p$i.log"; exit 6; }
  done
  cd "$GRAFT_REPO_ROOT"
  python tools/pmc_summary.py $O > $O/summary.txt 2>&1; cat $O/summary.txt
fi
