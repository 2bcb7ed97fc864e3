# Round-end check: PMC of every config (-> profiles/pmc_kernels.json on the
# box, so the bench lines carry traffic / issue), GPU tests, smoke, every
# bench line (incl. the driver's, N = 6 / 12, eager and closed loop), rocprof
# kernel stats of the H, C4, eager and closed-loop commands.
# Usage: bash tools/gpu_final.sh TAG [nopmc]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=${1:-final}; O=gpurun_out/$T; mkdir -p $O
if [ "$2" != nopmc ]; then
  timeout -k 10 1000 bash tools/pmc_all.sh $T > $O/pmc_all.log 2>&1 || { tail -20 $O/pmc_all.log; exit 1; }
  cp gpurun_out/profiles_new/pmc_kernels.json profiles/pmc_kernels.json
  mkdir -p $O/pmc && cp -r gpurun_out/profiles_new/pmc_kernels.json $O/pmc/ && for d in gpurun_out/${T}_pmc_*; do mkdir -p $O/pmc/$(basename $d) && cp $d/summary.txt $O/pmc/$(basename $d)/; done
  echo "pmc collected"
fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 2; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_h.json 2> $O/bench_h.err || { tail -20 $O/bench_h.err; exit 4; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_h_driver.json 2> $O/bench_h_driver.err || { tail -20 $O/bench_h_driver.err; exit 4; }
for c in c2 c3 c4; do
  timeout -k 10 300 python bench.py --config $c --cpu-seconds 10 > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 5; }
done
for n in 6 12; do
  timeout -k 10 300 python bench.py --n-agents $n --no-cpu-baseline > $O/bench_h_n$n.json 2> $O/bench_h_n$n.err || { tail -20 $O/bench_h_n$n.err; exit 5; }
done
for m in eager policy; do
  timeout -k 10 300 python bench.py --$m --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_h_$m.json 2> $O/bench_h_$m.err || { tail -20 $O/bench_h_$m.err; exit 5; }
done
for n in h h_driver c2 c3 c4 h_n6 h_n12 h_eager h_policy; do
  python -c "import json; d=json.load(open('$O/bench_$n.json')); r=d['roofline'] or {}; print('$n', d['value'], d['ms_per_step'], r.get('bound'), r.get('frac'), r.get('issue_frac'), r.get('traffic'), (r.get('pmc') or {}).get('status'))"
done
cd /tmp
for c in h c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_$c" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config $c --no-cpu-baseline > "$GRAFT_REPO_ROOT/$O/prof_$c.log" 2>&1 || exit 6
done
for m in eager policy; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_h_$m" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --$m --steps 200 --warmup 20 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$O/prof_h_$m.log" 2>&1 || exit 7
done
echo done
