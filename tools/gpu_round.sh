# Round measurement: GPU tests, smoke, the default bench line (with CPU
# baseline), the other BASELINE configs, and rocprofv3 kernel stats of the
# default bench command. Usage: bash tools/gpu_round.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r1}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -m pytest tests -m gpu -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_h.json 2> $O/bench_h.err || { tail -20 $O/bench_h.err; exit 4; }
cat $O/bench_h.json
for c in c2 c3 c4; do
  timeout -k 10 300 python bench.py --config $c --cpu-seconds 10 > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 5; }
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1 || exit 6
cd "$GRAFT_REPO_ROOT" && for c in c2 c3 c4; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_$c" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --config $c --no-cpu-baseline > "$GRAFT_REPO_ROOT/$O/prof_$c.log" 2>&1 || exit 7
done
cd "$GRAFT_REPO_ROOT" && timeout -k 10 300 python bench.py --unfused --no-cpu-baseline > $O/bench_h_unfused.json 2> $O/bench_h_unfused.err || exit 8
echo done
