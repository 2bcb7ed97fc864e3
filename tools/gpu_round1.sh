set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
echo "== pytest gpu"; timeout -k 10 400 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/r1_pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/r1_pytest_gpu.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo "== smoke"; timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1_smoke.log 2>&1 || { cat gpurun_out/r1_smoke.log | tail -20; exit 3; }
tail -2 gpurun_out/r1_smoke.log
echo "== bench"; timeout -k 10 300 python bench.py --cpu-seconds 10 > gpurun_out/r1_bench.json 2> gpurun_out/r1_bench.err || { tail -30 gpurun_out/r1_bench.err; exit 4; }
cat gpurun_out/r1_bench.json; tail -3 gpurun_out/r1_bench.err
echo "== bench no events"; timeout -k 10 300 python bench.py --no-cpu-baseline --no-timing-events > gpurun_out/r1_bench_noev.json 2> gpurun_out/r1_bench_noev.err || exit 5
cat gpurun_out/r1_bench_noev.json
echo "== rocprof"; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r1_prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --steps 300 --warmup 50 > "$GRAFT_REPO_ROOT/gpurun_out/r1_prof.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/r1_prof.log"; exit 6; }
find "$GRAFT_REPO_ROOT/gpurun_out/r1_prof" -name "*stats*" | head
