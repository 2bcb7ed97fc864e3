# Bench lines only: the default (headline) line, the driver's short line and C4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${1:-r2_n}; mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_h.json 2> $O/bench_h.err || { tail -20 $O/bench_h.err; exit 4; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_h_driver.json 2> $O/bench_h_driver.err || { tail -20 $O/bench_h_driver.err; exit 5; }
timeout -k 10 300 python bench.py --config c4 --cpu-seconds 10 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 6; }
python - $O <<'PY'
import json, sys
for n in ("bench_h", "bench_h_driver", "bench_c4"):
    d = json.load(open(f"{sys.argv[1]}/{n}.json"))
    r = d["roofline"]
    print(n, d["value"], d["ms_per_step"], r["bound"], r["frac"], r.get("issue_frac"), r["pmc"]["status"] if "pmc" in r else "")
PY
