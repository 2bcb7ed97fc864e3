# PMC passes (tools/pmc.sh) for the BASELINE bench configs, merged into
# profiles/pmc_traffic.json for bench.py's roofline.traffic.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/pmc.sh pmc_h --config h > /dev/null || exit 1
bash tools/pmc.sh pmc_c2 --config c2 > /dev/null || exit 1
bash tools/pmc.sh pmc_c3 --config c3 > /dev/null || exit 1
bash tools/pmc.sh pmc_c4 --config c4 > /dev/null || exit 1
PMC_GRAPH=1 bash tools/pmc.sh pmc_h_lag --config h > /dev/null || exit 1
PMC_GRAPH=1 bash tools/pmc.sh pmc_c2_lag --config c2 > /dev/null || exit 1
mkdir -p gpurun_out/profiles_new
python tools/pmc_traffic.py gpurun_out/profiles_new/pmc_traffic.json \
  h:navigation:N24:B8192=gpurun_out/pmc_h c2:navigation:N3:B4096=gpurun_out/pmc_c2 \
  c3:navigation:N96:B1024=gpurun_out/pmc_c3 c4:mixed:N24:B8192=gpurun_out/pmc_c4 \
  lag@h:navigation:N24:B8192=gpurun_out/pmc_h_lag lag@c2:navigation:N3:B4096=gpurun_out/pmc_c2_lag
