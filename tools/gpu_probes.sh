# Round-2 evidence for DESIGN.md §5 / §8: instruction latency and issue rate
# (tools/probe_latency.hip), headline lagged-step time vs batch size
# (tools/ablate.py), graph launch + final-emit fixed cost
# (tools/probe_graph_launch.py). Usage: bash tools/gpu_probes.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
timeout -k 5 60 ./tools/probe_latency > $O/probe_latency.txt 2>&1 || exit 1
for b in 1024 2048 4096 6144 7168 8192 9216 12288 16384; do
  ABL_B=$b timeout -k 10 100 python tools/ablate.py 2>/dev/null >> $O/batch_scaling.jsonl || exit 2
done
B=64 timeout -k 10 100 python tools/probe_graph_launch.py > $O/graph_launch.txt 2>&1 || exit 3
B=8192 timeout -k 10 100 python tools/probe_graph_launch.py >> $O/graph_launch.txt 2>&1 || exit 3
cat $O/probe_latency.txt $O/graph_launch.txt
python -c "
import json
for l in open('$O/batch_scaling.jsonl'):
    d = json.loads(l); print(d['B'], round(d['lag_step_ms']*1e3, 2), round(d['step_ms']*1e3, 2), round(d['emit_ms']*1e3, 2))"
