# The whole round-end measurement package on one code object, in one call:
# PMC of every bench configuration (-> profiles/pmc_kernels.json on the box,
# copied to gpurun_out/profiles_new/), GPU tests, smoke, every bench line and
# rocprof kernel stats. Usage: bash tools/gpu_package.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=${1:-pk}; O=gpurun_out/$T; mkdir -p $O/pmc
run() { timeout -k 10 280 bash tools/pmc.sh "$@" > $O/$1.log 2>&1 || { tail -20 $O/$1.log; exit 1; }
        mkdir -p $O/pmc/$1 && cp gpurun_out/$1/summary.txt $O/pmc/$1/; }
PMC_ROLL=1 run ${T}_pmc_h_roll --config h
PMC_ROLL=1 run ${T}_pmc_c2_roll --config c2
PMC_ROLL=1 run ${T}_pmc_c3_roll --config c3
PMC_ROLL=1 run ${T}_pmc_c4_roll --config c4
PMC_ROLL=1 run ${T}_pmc_n6_roll --n-agents 6
PMC_ROLL=1 run ${T}_pmc_n12_roll --n-agents 12
run ${T}_pmc_h --config h
run ${T}_pmc_c2 --config c2
run ${T}_pmc_c4 --config c4
PMC_GRAPH=1 run ${T}_pmc_h_lag --config h
PMC_GRAPH=1 run ${T}_pmc_c4_lag --config c4
rm -f profiles/pmc_kernels.json
python tools/pmc_traffic.py profiles/pmc_kernels.json \
  roll@h:navigation:N24:B8192=gpurun_out/${T}_pmc_h_roll roll@c2:navigation:N3:B4096=gpurun_out/${T}_pmc_c2_roll \
  roll@c3:navigation:N96:B1024=gpurun_out/${T}_pmc_c3_roll roll@c4:mixed:N24:B8192=gpurun_out/${T}_pmc_c4_roll \
  roll@h:navigation:N6:B8192=gpurun_out/${T}_pmc_n6_roll roll@h:navigation:N12:B8192=gpurun_out/${T}_pmc_n12_roll \
  h:navigation:N24:B8192=gpurun_out/${T}_pmc_h c2:navigation:N3:B4096=gpurun_out/${T}_pmc_c2 \
  c4:mixed:N24:B8192=gpurun_out/${T}_pmc_c4 lag@h:navigation:N24:B8192=gpurun_out/${T}_pmc_h_lag \
  lag@c4:mixed:N24:B8192=gpurun_out/${T}_pmc_c4_lag > /dev/null || exit 1
mkdir -p gpurun_out/profiles_new && cp profiles/pmc_kernels.json gpurun_out/profiles_new/pmc_kernels.json && cp profiles/pmc_kernels.json $O/pmc/
echo "pmc collected"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 2; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
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
