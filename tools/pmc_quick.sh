# Quick PMC passes of one config's rollout (a 100-step launch), per wave-step
# instruction counts and per-step HBM bytes, for A/B of library builds.
# Usage: PMC_CONFIG=h|c2|c3|c4 PMC_SET="inst traffic" bash tools/pmc_quick.sh TAG [LIB ...]
# (LIB: a path under gs-marl_amd/gsmarl_amd/lib, default the product library)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
CFG=${PMC_CONFIG:-h}
ARGS=""; [ "$CFG" != h ] && ARGS="--config $CFG"
for L in ${@:-libgsm.so}; do
  n=$(basename $L .so)
  for s in ${PMC_SET:-inst}; do
    case $s in
      inst) passes=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE") ;;
      traffic) passes=("SQ_WAVES FETCH_SIZE" "SQ_WAVES WRITE_SIZE") ;;
      *) echo "unknown set $s"; exit 9 ;;
    esac
    i=0
    for grp in "${passes[@]}"; do
      i=$((i + 1))
      ( cd /tmp && GSM_LIB_PATH=$GRAFT_REPO_ROOT/gs-marl_amd/gsmarl_amd/lib/$L timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $O/$n/$s$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-kernel-timing --settle-ms 0 --warmup 0 --no-align --steps 100 $ARGS > $O/$n.$s$i.log 2>&1 ) || { echo "fail $n $s$i"; tail -5 $O/$n.$s$i.log; exit 1; }
    done
  done
  python3 - $O/$n "$n $CFG" <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gsm_roll" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in acc.items()}
w = m.get("SQ_WAVES", 1) * 100
out = [sys.argv[2], "per wave-step:"]
for k, nm in (("SQ_INSTS_SALU", "SALU"), ("SQ_INSTS_VALU", "VALU"), ("SQ_INSTS_LDS", "LDS")):
    if k in m:
        out += [nm, round(m[k] / w, 1)]
if "GRBM_GUI_ACTIVE" in m:
    out += ["launch cycles/step", round(m["GRBM_GUI_ACTIVE"] / 8 / 100)]
if "FETCH_SIZE" in m:   # KiB, x2 on gfx950 (MI355X_MICROARCH.md)
    out += ["HBM read MB/step", round(2 * m["FETCH_SIZE"] * 1024 / 100 / 1e6, 2)]
if "WRITE_SIZE" in m:
    out += ["write MB/step", round(m["WRITE_SIZE"] * 1024 / 100 / 1e6, 2)]
print(*out)
PY
done
