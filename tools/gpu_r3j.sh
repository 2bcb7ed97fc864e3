set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r3_m; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_roll_ragged.py tests/test_gpu_roll_concurrency.py -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_rr.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|placement" $O/pytest_rr.log | tail -25
[ $rc -eq 0 ] || { grep -B2 -A30 "Error\|assert" $O/pytest_rr.log | head -60; exit 2; }
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 4; }
python -c "import json;d=json.load(open('$O/bench_c4.json'));r=d['roofline'];print('c4', d['value'], d['ms_per_step'], r['kernel'], r['mean_launch_us'])"
GSM_ROLL_PLACE=0 timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --no-kernel-timing > $O/bench_c4_noplace.json 2> $O/bench_c4_noplace.err || { tail -20 $O/bench_c4_noplace.err; exit 5; }
python -c "import json;d=json.load(open('$O/bench_c4_noplace.json'));print('c4 no placement', d['value'], d['ms_per_step'])"
GSM_LIB_PATH=$PWD/gs-marl_amd/gsmarl_amd/lib/ablate/stamps.so timeout -k 10 240 python tools/stamps_c4_roll.py > $O/stamps.json 2> $O/stamps.err || { tail -20 $O/stamps.err; exit 6; }
python -c "
import json;d=json.load(open('$O/stamps.json'))
for k in ('placement_decisions','placement_wait_us_max','placement_wait_us_p50','launch_ms_events','span_us','end_p50_us','phase_cycles_mean_per_step','simd_work_cycles_per_step','cold_solves'): print(k, d[k])
"
