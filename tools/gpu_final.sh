# Round-end check: GPU tests, smoke, every bench line, rocprof stats of the H and C4 commands.
# Usage: bash tools/gpu_final.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=${1:-r2_final}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 2; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_h.json 2> $O/bench_h.err || { tail -20 $O/bench_h.err; exit 4; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_h_driver.json 2> $O/bench_h_driver.err || { tail -20 $O/bench_h_driver.err; exit 4; }
for c in c2 c3 c4; do
  timeout -k 10 300 python bench.py --config $c --cpu-seconds 10 > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 5; }
done
for n in h h_driver c2 c3 c4; do
  python -c "import json; d=json.load(open('$O/bench_$n.json')); r=d['roofline']; print('$n', d['value'], d['ms_per_step'], r['bound'], r['frac'], r['issue_frac'], r['traffic'], r['pmc']['status'])"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_h" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/$O/prof_h.log" 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_c4" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config c4 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$O/prof_c4.log" 2>&1 || exit 7
echo done
