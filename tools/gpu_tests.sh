# GPU tests + smoke + bench lines of every BASELINE config (no CPU baseline)
# and the driver's short headline line. Usage: bash tools/gpu_tests.sh TAG [pytest -k expr]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-t}
O=gpurun_out/$TAG
mkdir -p $O
K=${2:+-k "$2"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider $K > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|error" $O/pytest_gpu.log | tail -3; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_gpu.log | head -80; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_h_driver.json 2> $O/bench_h_driver.err || { tail -20 $O/bench_h_driver.err; exit 4; }
for c in h c2 c3 c4; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 4; }
done
for n in h_driver h c2 c3 c4; do
  python -c "import json;d=json.load(open('$O/bench_$n.json'));r=d['roofline'];print('$n',d['value'],'us/step',round(d['ms_per_step']*1e3,2),r['kernel'][:22],r['mean_launch_us'],'us frac',r['frac'],'pmc',r['pmc']['status'][:20])"
done
# the reference's zero-shot navigation sizes (readme.md:75): rollouts at N = 6, 12
for n in 6 12; do
  timeout -k 10 300 python bench.py --n-agents $n --no-cpu-baseline > $O/bench_h_n$n.json 2> $O/bench_h_n$n.err || { tail -20 $O/bench_h_n$n.err; exit 5; }
  python -c "import json;d=json.load(open('$O/bench_h_n$n.json'));r=d['roofline'];print('h n$n',d['value'],'us/step',round(d['ms_per_step']*1e3,2),r['kernel'][:22],r['mean_launch_us'])"
done
