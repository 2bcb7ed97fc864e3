# Rollout iteration: rollout tests, the launch probe (tools/probe_launch.py) for
# the library and an optional variant build, the driver's short bench line.
# Usage: bash tools/gpu_probe_launch.sh TAG [variant-name]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-probe}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_roll.py tests/test_gpu_rollout.py tests/test_gpu_oracle_direct.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_roll.log 2>&1 || { tail -40 $O/pytest_roll.log; exit 2; }
tail -1 $O/pytest_roll.log
for rep in 1 2; do
  timeout -k 10 120 python tools/probe_launch.py > $O/probe_lib_$rep.json || exit 3
  cat $O/probe_lib_$rep.json
  if [ -n "$2" ]; then
    GSM_LIB_PATH=gs-marl_amd/gsmarl_amd/lib/ablate/$2.so timeout -k 10 120 python tools/probe_launch.py > $O/probe_$2_$rep.json || exit 3
    cat $O/probe_$2_$rep.json
  fi
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_h_driver.json 2> $O/bench_h_driver.err || { tail -20 $O/bench_h_driver.err; exit 4; }
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_h.json 2> $O/bench_h.err || { tail -20 $O/bench_h.err; exit 4; }
for n in h_driver h; do python -c "import json;d=json.load(open('$O/bench_$n.json'));r=d['roofline'];print('$n', d['value'], d['ms_per_step'], r['mean_launch_us'])"; done
