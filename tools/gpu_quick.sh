# Bench lines for the BASELINE configs and a rocprofv3 kernel-trace summary of
# the default (headline) bench command. Usage: bash tools/gpu_quick.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-q}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python bench.py --cpu-seconds 10 > $O/bench_h.json 2> $O/bench_h.err || { tail -20 $O/bench_h.err; exit 4; }
for c in c2 c3 c4; do
  timeout -k 10 300 python bench.py --config $c --cpu-seconds 10 > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 5; }
done
timeout -k 10 300 python bench.py --unfused --no-cpu-baseline > $O/bench_h_unfused.json 2> $O/bench_h_unfused.err || exit 8
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1 || exit 6
cd "$GRAFT_REPO_ROOT"
for c in h c2 c3 c4 h_unfused; do
  python -c "import json;d=json.load(open('$O/bench_$c.json'));r=d['roofline'];print('$c',d['value'],'us/step',round(d['ms_per_step']*1e3,2),r['kernel'],r['mean_launch_us'],'us',r['achieved'],'GB/s frac',r['frac'],'other',r['other_kernel']['mean_launch_us'])"
done
find $O/prof -name "*kernel_stats.csv" -exec head -4 {} \; | cut -c1-220
