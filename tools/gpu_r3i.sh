set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r3_i; mkdir -p $O
timeout -k 10 300 python tools/probe_c4_balance.py > $O/balance.jsonl 2> $O/balance.err || { tail -20 $O/balance.err; exit 2; }
cat $O/balance.jsonl
for m in eager policy; do
  timeout -k 10 200 python bench.py --$m --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_h_$m.json 2> $O/bench_h_$m.err || { tail -20 $O/bench_h_$m.err; exit 3; }
  python -c "import json;d=json.load(open('$O/bench_h_$m.json'));print('$m', d['value'], d['ms_per_step'])"
done
