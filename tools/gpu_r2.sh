# Round-2 measurement: GPU tests, smoke, bench lines for every BASELINE config
# (headline with the CPU baseline), rocprofv3 kernel stats of each bench
# command, the --gpus N launcher's refusal on a 1-GPU box, and (PMC=1) the
# PMC passes behind roofline.traffic / valu_frac. Usage: bash tools/gpu_r2.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r2}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
if [ -n "$PMC" ]; then
  bash tools/pmc_all.sh $TAG || exit 9
  cp gpurun_out/profiles_new/pmc_kernels.json profiles/pmc_kernels.json
fi
timeout -k 10 300 python bench.py > $O/bench_h.json 2> $O/bench_h.err || { tail -20 $O/bench_h.err; exit 4; }
for c in c2 c3 c4; do
  timeout -k 10 300 python bench.py --config $c --cpu-seconds 10 > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 5; }
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_h_driver.json 2> $O/bench_h_driver.err || exit 8
timeout -k 10 300 python bench.py --no-roll --no-cpu-baseline > $O/bench_h_noroll.json 2> $O/bench_h_noroll.err || exit 8
timeout -k 10 300 python bench.py --config c3 --no-roll --no-cpu-baseline > $O/bench_c3_noroll.json 2> $O/bench_c3_noroll.err || exit 8
timeout -k 10 300 python bench.py --config c2 --no-roll --no-cpu-baseline > $O/bench_c2_noroll.json 2> $O/bench_c2_noroll.err || exit 8
timeout -k 10 120 python bench.py --gpus 2 --steps 5 > $O/bench_gpus2.out 2>&1; echo "bench --gpus 2 on one GPU: exit $?" >> $O/bench_gpus2.out
for c in h c2 c3 c4; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_$c" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --config $c --no-cpu-baseline > "$GRAFT_REPO_ROOT/$O/prof_$c.log" 2>&1 || exit 7
done
cd "$GRAFT_REPO_ROOT"
for c in h c2 c3 c4 h_driver h_noroll c2_noroll c3_noroll; do
  python -c "import json;d=json.load(open('$O/bench_$c.json'));r=d['roofline'];print('$c',d['value'],'us/step',round(d['ms_per_step']*1e3,2),r['kernel'],r['mean_launch_us'],'us frac',r['frac'],'valu',r['valu_frac'],'issue',r.get('issue_frac'),'traffic',r['traffic'],'bounds',d['timed_region']['episode_boundaries'])"
done
tail -2 $O/bench_gpus2.out
echo done
