# Rollout iteration: rollout tests, the launch probe of the library and of
# variants (tools/gpu_ablate.sh), the driver's short line with and without
# settling. Usage: bash tools/gpu_iter.sh TAG [variant ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-iter}; shift; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_roll.py tests/test_gpu_rollout.py tests/test_gpu_oracle_direct.py tests/test_gpu_roll_concurrency.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_roll.log 2>&1 || { tail -40 $O/pytest_roll.log; exit 2; }
tail -1 $O/pytest_roll.log
bash tools/gpu_ablate.sh $T "$@" || exit 3
for ms in 0 20 0 20; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing --settle-ms $ms > $O/d.json 2>$O/d.err || { tail $O/d.err; exit 4; }
  python -c "import json;d=json.load(open('$O/d.json'));print('driver settle $ms ms', d['ms_per_step'])"
done
