# quick iteration: GPU tests, then bench (events + no events) and a rocprof kernel-trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-it}
timeout -k 10 400 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -4 gpurun_out/${TAG}_pytest.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 4; }
cat gpurun_out/${TAG}_bench.json; grep kernels gpurun_out/${TAG}_bench.err
timeout -k 10 300 python bench.py --no-cpu-baseline --no-timing-events > gpurun_out/${TAG}_bench_noev.json 2>/dev/null || exit 5
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_noev.json'));print('noev value',d['value'],'ms/step',d['ms_per_step'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-timing-events > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" 2>&1 || exit 6
head -3 "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof/run_kernel_stats.csv"
