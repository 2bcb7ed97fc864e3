# Spread of the driver's own bench command over fresh processes on one box:
# R runs of `bench.py --gpus 1 --steps 20 --warmup 5` (no CPU baseline), plain
# and pinned to one host core (taskset, before any GPU use), alternating.
# Usage: bash tools/driver_spread.sh TAG [R]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=$1; R=${2:-6}
O=gpurun_out/$T; mkdir -p $O
for i in $(seq 1 $R); do
  timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/plain_$i.json 2> $O/plain_$i.err || exit 1
  timeout -k 10 120 taskset -c 3 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/pin_$i.json 2> $O/pin_$i.err || exit 1
done
python3 - $O <<'PY'
import json, glob, sys
for k in ("plain", "pin"):
    v = []
    for f in sorted(glob.glob(f"{sys.argv[1]}/{k}_*.json")):
        d = json.loads(open(f).read().strip().splitlines()[-1])
        t = d["timed_region"]
        v.append((round(d["ms_per_step"] * 1e3, 2), t.get("graph_device_us"), t.get("host_us"), t.get("fill_us")))
    print(k, v)
PY
