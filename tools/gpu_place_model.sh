# C4 rollout time per step under placement cost models (GSM_PLACE_MODEL="a,b,c,d":
# polygon/line a + b N, navigation c + d N), alternating on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-place}; shift; mkdir -p $O
for rep in 1 2; do for m in "$@"; do
  GSM_PLACE_MODEL=$m timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline --no-kernel-timing --steps 200 > $O/b.json 2>$O/b.err || { tail $O/b.err; exit 3; }
  python -c "import json;d=json.load(open('$O/b.json'));print('model $m', d['ms_per_step'])"
done; done
