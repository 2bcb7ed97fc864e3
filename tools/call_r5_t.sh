# Round-5 call: the count-based, rank-aligned settle loop: the driver command
# three times, the h and eager lines, and the launcher's single-rank torchrun
# form of the driver command.
cd $GRAFT_REPO_ROOT; O=gpurun_out/cx; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$r.json 2> $O/driver_$r.err || { tail -20 $O/driver_$r.err; exit 3; }
  python3 -c "import json; d=json.load(open('$O/driver_$r.json')); print('driver', d['ms_per_step'], d['timed_region']['settle_steps'], d['timed_region']['host_us'], d['timed_region']['fill_us'])"
done
timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/driver_trun.json 2> $O/driver_trun.err || { tail -20 $O/driver_trun.err; exit 4; }
python3 -c "import json; d=json.loads(open('$O/driver_trun.json').read().strip().splitlines()[-1]); print('torchrun', d['ms_per_step'], d['n_gpus'])"
for l in h eager; do bash tools/gpu.sh lines cx $l || exit 5; done
