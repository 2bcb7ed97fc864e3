# quick iteration: GPU tests, bench for the headline + C2/C3 configs, and a
# rocprof kernel-trace of the default bench command
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-it}
timeout -k 10 400 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -4 gpurun_out/${TAG}_pytest.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-h c2 c3}; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err || { tail -20 gpurun_out/${TAG}_bench_$c.err; exit 4; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$c.json'));r=d['roofline'];print('$c',d['value'],'ms/step',d['ms_per_step'],r['kernel'],r['mean_launch_us'],'us',r['achieved'],'GB/s', 'other',r['other_kernel']['mean_launch_us'])"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" 2>&1 || exit 6
head -3 "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof/run_kernel_stats.csv" | cut -c1-200
