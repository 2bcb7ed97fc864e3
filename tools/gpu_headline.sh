# Headline measurement package in one call: PMC of the headline rollout (->
# profiles/pmc_kernels.json on the box, so the bench line carries traffic /
# issue), GPU tests, smoke, the default and the driver's bench lines, rocprof
# kernel stats of the default command. Usage: bash tools/gpu_headline.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=${1:-hl}; O=gpurun_out/$T; mkdir -p $O
PMC_ROLL=1 timeout -k 10 280 bash tools/pmc.sh ${T}_pmc_h_roll --config h > $O/pmc_h_roll.log 2>&1 || { tail -20 $O/pmc_h_roll.log; exit 1; }
mkdir -p gpurun_out/profiles_new && rm -f gpurun_out/profiles_new/pmc_kernels.json
python tools/pmc_traffic.py gpurun_out/profiles_new/pmc_kernels.json \
  roll@h:navigation:N24:B8192=gpurun_out/${T}_pmc_h_roll > /dev/null || exit 1
cp gpurun_out/profiles_new/pmc_kernels.json profiles/pmc_kernels.json
mkdir -p $O/pmc/${T}_pmc_h_roll && cp gpurun_out/profiles_new/pmc_kernels.json $O/pmc/ && cp gpurun_out/${T}_pmc_h_roll/summary.txt $O/pmc/${T}_pmc_h_roll/
echo "pmc collected"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 2; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_h.json 2> $O/bench_h.err || { tail -20 $O/bench_h.err; exit 4; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_h_driver.json 2> $O/bench_h_driver.err || { tail -20 $O/bench_h_driver.err; exit 4; }
for n in h h_driver; do
  python -c "import json; d=json.load(open('$O/bench_$n.json')); r=d['roofline'] or {}; print('$n', d['value'], d['ms_per_step'], r.get('bound'), r.get('frac'), r.get('issue_frac'), r.get('traffic'), (r.get('pmc') or {}).get('status'))"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_h" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/$O/prof_h.log" 2>&1 || exit 6
echo done
