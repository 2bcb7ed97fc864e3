# C4 ragged rollout: step time and HBM traffic (FETCH_SIZE / WRITE_SIZE of one
# 100-step launch) per hand-off depth. Usage: bash tools/gpu_c4_depth.sh TAG [depth ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=${1:-c4d}; shift; O=gpurun_out/$T; mkdir -p $O
for d in "${@:-2 3 4}"; do
  GSM_ROLL_DEPTH=$d timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $O/bench_d$d.json 2> $O/bench_d$d.err || { tail -20 $O/bench_d$d.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_d$d.json'));print('depth $d', d['ms_per_step'], d['roofline']['mean_launch_us'])"
  for grp in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && GSM_ROLL_DEPTH=$d timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$GRAFT_REPO_ROOT/$O/d${d}_$grp" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --config c4 --no-cpu-baseline --no-kernel-timing --settle-ms 0 --warmup 0 --no-align --steps 100 > "$GRAFT_REPO_ROOT/$O/d${d}_$grp.log" 2>&1 ) || { echo "pmc $d $grp failed"; exit 2; }
  done
  python - "$O" "$d" <<'EOF'
import csv, glob, sys
o, d = sys.argv[1], sys.argv[2]
for grp in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{o}/d{d}_{grp}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "roll_ragged" in r.get("Kernel_Name", ""):
                print(f"depth {d} {grp} {float(r['Counter_Value']):.0f} KiB per launch")
EOF
done
