set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r2_n; mkdir -p $O
for c in c4 c2 c3; do
timeout -k 10 300 python bench.py --config $c --cpu-seconds 10 > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 6; }
python -c "import json,sys; d=json.load(open('$O/bench_$c.json')); r=d['roofline']; print('$c', d['value'], d['ms_per_step'], r['bound'], r['frac'], r['issue_frac'])"
done
