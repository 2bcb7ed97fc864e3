# One PMC pass (instruction counts) of the headline rollout, per wave-step:
# SALU, VALU, LDS instructions and the launch's cycles, for A/B of instruction
# budgets between library builds. Usage: bash tools/pmc_quick.sh TAG [LIB ...]
# (LIB: a path under gs-marl_amd/gsmarl_amd/lib, default the product library)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
for L in ${@:-libgsm.so}; do
  n=$(basename $L .so)
  ( cd /tmp && GSM_LIB_PATH=$GRAFT_REPO_ROOT/gs-marl_amd/gsmarl_amd/lib/$L timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/$n -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-kernel-timing --settle-ms 0 --warmup 0 --no-align --steps 100 > $O/$n.log 2>&1 ) || { echo "fail $n"; tail -5 $O/$n.log; exit 1; }
  python3 - $O/$n $n <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gsm_roll" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in acc.items()}
w = m.get("SQ_WAVES", 1) * 100
print(sys.argv[2], "per wave-step: SALU", round(m["SQ_INSTS_SALU"] / w, 1), "VALU", round(m["SQ_INSTS_VALU"] / w, 1),
      "LDS", round(m["SQ_INSTS_LDS"] / w, 1), "launch cycles/step", round(m["GRBM_GUI_ACTIVE"] / 8 / 100))
PY
done
