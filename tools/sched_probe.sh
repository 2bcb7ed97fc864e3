cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/sched
for m in default spin yield block; do
  timeout -k 10 180 python3 tools/probe_launch.py --sched $m > gpurun_out/sched/$m.json 2> gpurun_out/sched/$m.err || exit 1
done
timeout -k 10 180 python3 tools/probe_launch.py --sched spin --sched-when late > gpurun_out/sched/spin_late.json 2> gpurun_out/sched/spin_late.err || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/sched/driver_default.json 2>gpurun_out/sched/d.err || exit 1
GSM_TEST_SCHED=1 timeout -k 10 300 python3 -c "
import ctypes,sys,runpy
ctypes.CDLL('libamdhip64.so.7')
" || exit 1
cat gpurun_out/sched/*.json
