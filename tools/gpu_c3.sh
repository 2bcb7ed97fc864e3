# Tile (C3) iteration: tile-shape GPU tests, C3 bench lines (lagged and two-kernel chain).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-c3}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_rollout.py tests/test_gpu_degenerate.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest.log | head -60; exit $rc; }
for v in "" "--unfused"; do
  timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline $v > $O/c3$v.json 2>$O/c3$v.err || { tail $O/c3$v.err; exit 4; }
  python -c "import json;d=json.load(open('$O/c3$v.json'));r=d['roofline'];print('c3$v',d['value'],round(d['ms_per_step']*1e3,2),r['kernel'],r['mean_launch_us'],r['other_kernel']['mean_launch_us'])"
done
