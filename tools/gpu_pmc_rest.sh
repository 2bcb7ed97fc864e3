# PMC of the remaining bench configurations on the current code object, merged
# into profiles/pmc_kernels.json (copied to gpurun_out/profiles_new/): the
# navigation N = 6 / 12 rollouts, the per-step chains (lagged step kernel) and
# the eager step / emit kernels of H, C2, C4; then the N = 6 / 12 bench lines.
# Usage: bash tools/gpu_pmc_rest.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=${1:-pr}; O=gpurun_out/$T; mkdir -p $O/pmc
run() { timeout -k 10 280 bash tools/pmc.sh "$@" > $O/$1.log 2>&1 || { tail -20 $O/$1.log; exit 1; }
        mkdir -p $O/pmc/$1 && cp gpurun_out/$1/summary.txt $O/pmc/$1/; }
PMC_ROLL=1 run ${T}_pmc_n6_roll --n-agents 6
PMC_ROLL=1 run ${T}_pmc_n12_roll --n-agents 12
run ${T}_pmc_h --config h
run ${T}_pmc_c2 --config c2
run ${T}_pmc_c4 --config c4
PMC_GRAPH=1 run ${T}_pmc_h_lag --config h
PMC_GRAPH=1 run ${T}_pmc_c4_lag --config c4
python tools/pmc_traffic.py profiles/pmc_kernels.json \
  roll@h:navigation:N6:B8192=gpurun_out/${T}_pmc_n6_roll roll@h:navigation:N12:B8192=gpurun_out/${T}_pmc_n12_roll \
  h:navigation:N24:B8192=gpurun_out/${T}_pmc_h c2:navigation:N3:B4096=gpurun_out/${T}_pmc_c2 \
  c4:mixed:N24:B8192=gpurun_out/${T}_pmc_c4 lag@h:navigation:N24:B8192=gpurun_out/${T}_pmc_h_lag \
  lag@c4:mixed:N24:B8192=gpurun_out/${T}_pmc_c4_lag > /dev/null || exit 1
mkdir -p gpurun_out/profiles_new && cp profiles/pmc_kernels.json gpurun_out/profiles_new/pmc_kernels.json
python -c "import json; print(sorted(json.load(open('profiles/pmc_kernels.json'))['entries']))"
for n in 6 12; do
  timeout -k 10 300 python bench.py --n-agents $n --no-cpu-baseline > $O/bench_h_n$n.json 2> $O/bench_h_n$n.err || { tail -20 $O/bench_h_n$n.err; exit 5; }
  python -c "import json; d=json.load(open('$O/bench_h_n$n.json')); r=d['roofline']; print('n$n', d['value'], d['ms_per_step'], r.get('bound'), r.get('frac'), r.get('issue_frac'), r.get('traffic'), (r.get('pmc') or {}).get('status'))"
done
