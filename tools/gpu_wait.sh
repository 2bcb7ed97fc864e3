# Host completion latency: the launch probe and the driver's short line under
# HIP's default wait and with ROC_ACTIVE_WAIT_TIMEOUT raised (the runtime
# spins on the completion signal instead of sleeping on an interrupt).
# Usage: bash tools/gpu_wait.sh TAG [timeout_us ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-wait}; shift; mkdir -p $O
for w in default "$@" default "$@"; do
  if [ $w = default ]; then E="env -u ROC_ACTIVE_WAIT_TIMEOUT"; else E="env ROC_ACTIVE_WAIT_TIMEOUT=$w"; fi
  $E timeout -k 10 120 python tools/probe_launch.py > $O/probe_$w.json || exit 3
  echo "wait $w $(cat $O/probe_$w.json)"
  $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing > $O/d_$w.json 2>$O/d_$w.err || { tail $O/d_$w.err; exit 4; }
  python -c "import json;d=json.load(open('$O/d_$w.json'));print('driver wait $w', d['ms_per_step'])"
done
