# The driver's short headline line, repeated, with and without settling
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-drv}; mkdir -p $O
for ms in 0 20 100 0 20 100; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing --settle-ms $ms > $O/d$ms.json 2>$O/d$ms.err || { tail $O/d$ms.err; exit 2; }
  python -c "import json;d=json.load(open('$O/d$ms.json'));print('settle $ms ms', d['ms_per_step'], d['timed_region']['settle_steps'])"
done
