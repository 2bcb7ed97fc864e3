# Headline with the fused rollout: tests, bench lines (rollout and lagged
# chain), rocprofv3 kernel-trace stats of the default bench, PMC of the
# rollout launch. Usage: bash tools/gpu_h_roll.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-hroll}
O=gpurun_out/$TAG
mkdir -p $O
bash tools/gpu_roll.sh $TAG || exit 3
timeout -k 10 300 python bench.py --cpu-seconds 10 > $O/bench_h.json 2> $O/bench_h.err || { tail -20 $O/bench_h.err; exit 4; }
timeout -k 10 300 python bench.py --no-roll --no-cpu-baseline > $O/bench_h_noroll.json 2> $O/bench_h_noroll.err || { tail -20 $O/bench_h_noroll.err; exit 5; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_h_driver.json 2> $O/bench_h_driver.err || { tail -20 $O/bench_h_driver.err; exit 5; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1 || exit 6
cd "$GRAFT_REPO_ROOT"
[ -n "$NO_PMC" ] || PMC_ROLL=1 bash tools/pmc.sh ${TAG}_pmc --config h > /dev/null || exit 7
for c in h h_noroll h_driver; do
  python -c "import json;d=json.load(open('$O/bench_$c.json'));r=d['roofline'];print('$c',d['value'],'us/step',round(d['ms_per_step']*1e3,2),r['kernel'],r['mean_launch_us'],'us',r['achieved'],'GB/s frac',r['frac'],'issue',r['issue_frac'])"
done
find $O/prof -name "*kernel_stats.csv" -exec head -6 {} \; | cut -c1-200
