set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r3_g; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_roll_ragged.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_rr.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest_rr.log | tail -25
[ $rc -eq 0 ] || { grep -B2 -A30 "Error\|assert" $O/pytest_rr.log | head -60; exit 2; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_roll.py tests/test_gpu_rollout.py tests/test_gpu_oracle_direct.py tests/test_gpu_ragged.py tests/test_golden.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_roll.log 2>&1 || { tail -40 $O/pytest_roll.log; exit 3; }
tail -1 $O/pytest_roll.log
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 4; }
python -c "import json;d=json.load(open('$O/bench_c4.json'));r=d['roofline'];print('c4', d['value'], d['ms_per_step'], r['kernel'], r['mean_launch_us'], d.get('assignment'))"
