set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r3_h; mkdir -p $O
GSM_LIB_PATH=$PWD/gs-marl_amd/gsmarl_amd/lib/ablate/stamps.so timeout -k 10 240 python tools/stamps_c4_roll.py > $O/stamps.json 2> $O/stamps.err || { tail -20 $O/stamps.err; exit 2; }
cat $O/stamps.json
for d in 2 3 6 8; do
  GSM_ROLL_DEPTH=$d timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline > $O/bench_c4_d$d.json 2> $O/bench_c4_d$d.err || { tail -20 $O/bench_c4_d$d.err; exit 3; }
  python -c "import json;d=json.load(open('$O/bench_c4_d$d.json'));print('depth $d', d['ms_per_step'], d['roofline']['mean_launch_us'])"
done
