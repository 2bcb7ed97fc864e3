# Launch probe (tools/probe_launch.py) of the library and of ablation variants
# built by tools/build_variant.sh (timing only: a variant's outputs are wrong).
# Usage: bash tools/gpu_ablate.sh TAG variant ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-abl}; shift; mkdir -p $O
timeout -k 10 120 python tools/probe_launch.py > $O/probe_lib.json || exit 3
cat $O/probe_lib.json
for v in "$@"; do
  GSM_LIB_PATH=$PWD/gs-marl_amd/gsmarl_amd/lib/ablate/$v.so timeout -k 10 120 python tools/probe_launch.py > $O/probe_$v.json || exit 3
  cat $O/probe_$v.json
done
