# C4 ragged rollout: PMC HBM traffic per step (FETCH_SIZE x2 + WRITE_SIZE, the
# gfx950 correction of MI355X_MICROARCH.md) at each edge-slab depth
# (GSM_ROLL_DEPTH). Usage: bash tools/pmc_c4_depth.sh TAG depth ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
for d in "${@:-2 4 8}"; do
  for c in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && GSM_ROLL_DEPTH=$d timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/d${d}_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c4 --no-cpu-baseline --no-kernel-timing --settle-ms 0 --warmup 0 --no-align --steps 100 > $O/d${d}_$c.log 2>&1 ) || { echo "fail d=$d $c"; tail -5 $O/d${d}_$c.log; exit 1; }
    python3 - $O/d${d}_$c $c $d <<'PY'
import csv, glob, sys
vals=[]
for f in glob.glob(sys.argv[1]+"/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "roll" in row.get("Kernel_Name","") and row["Counter_Name"]==sys.argv[2]:
            vals.append(float(row["Counter_Value"]))
m=sum(vals)/len(vals) if vals else 0
k = 2 if sys.argv[2]=="FETCH_SIZE" else 1
print("depth", sys.argv[3], sys.argv[2], "per step MB", round(k*m*1024/100/1e6, 2), "dispatches", len(vals))
PY
  done
done
