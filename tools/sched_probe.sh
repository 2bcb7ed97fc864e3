# Host wait mode of synchronize (hipSetDeviceFlags spin / yield / blocking, set
# before or after the first GPU use) against the launch + completion floor and
# a 20-step rollout replay (tools/probe_launch.py), plus the driver's command.
# Usage: bash tools/sched_probe.sh   (results in gpurun_out/sched/)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/sched
for m in default spin yield block; do
  timeout -k 10 180 python3 tools/probe_launch.py --sched $m > gpurun_out/sched/$m.json 2> gpurun_out/sched/$m.err || exit 1
done
timeout -k 10 180 python3 tools/probe_launch.py --sched spin --sched-when late > gpurun_out/sched/spin_late.json 2> gpurun_out/sched/spin_late.err || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/sched/driver_default.json 2> gpurun_out/sched/d.err
