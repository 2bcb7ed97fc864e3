# Ragged (C4) iteration: ragged GPU tests, C4 bench line, rocprof stats. Usage: bash tools/gpu_c4.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-c4}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ragged.py tests/test_gpu_degenerate.py -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|warm-start" $O/pytest_gpu.log | tail -6; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest_gpu.log | head -60; exit $rc; }
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 4; }
python -c "import json;d=json.load(open('$O/bench_c4.json'));r=d['roofline'];print('c4',d['value'],'us/step',round(d['ms_per_step']*1e3,2),r['kernel'],r['mean_launch_us'],'us frac',r['frac'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_c4" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --config c4 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$O/prof_c4.log" 2>&1 || exit 7
cd "$GRAFT_REPO_ROOT" && find $O/prof_c4 -name "*kernel_stats.csv" -exec head -4 {} \; | cut -c1-160
