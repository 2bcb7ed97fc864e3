# PMC passes (tools/pmc.sh) for the BASELINE bench configs, merged into
# gpurun_out/profiles_new/pmc_kernels.json (copy to profiles/ for bench.py's
# roofline.traffic / valu_frac; it carries the hash of the built code object).
# Usage: bash tools/pmc_all.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r2}
bash tools/pmc.sh ${T}_pmc_h --config h > /dev/null || exit 1
bash tools/pmc.sh ${T}_pmc_c2 --config c2 > /dev/null || exit 1
bash tools/pmc.sh ${T}_pmc_c3 --config c3 > /dev/null || exit 1
bash tools/pmc.sh ${T}_pmc_c4 --config c4 > /dev/null || exit 1
PMC_GRAPH=1 bash tools/pmc.sh ${T}_pmc_h_lag --config h > /dev/null || exit 1
PMC_GRAPH=1 bash tools/pmc.sh ${T}_pmc_c2_lag --config c2 > /dev/null || exit 1
PMC_GRAPH=1 bash tools/pmc.sh ${T}_pmc_c4_lag --config c4 > /dev/null || exit 1
PMC_ROLL=1 bash tools/pmc.sh ${T}_pmc_h_roll --config h > /dev/null || exit 1
PMC_ROLL=1 bash tools/pmc.sh ${T}_pmc_c3_roll --config c3 > /dev/null || exit 1
PMC_ROLL=1 bash tools/pmc.sh ${T}_pmc_c2_roll --config c2 > /dev/null || exit 1
PMC_ROLL=1 bash tools/pmc.sh ${T}_pmc_c4_roll --config c4 > /dev/null || exit 1
mkdir -p gpurun_out/profiles_new
rm -f gpurun_out/profiles_new/pmc_kernels.json
python tools/pmc_traffic.py gpurun_out/profiles_new/pmc_kernels.json \
  h:navigation:N24:B8192=gpurun_out/${T}_pmc_h c2:navigation:N3:B4096=gpurun_out/${T}_pmc_c2 \
  c3:navigation:N96:B1024=gpurun_out/${T}_pmc_c3 c4:mixed:N24:B8192=gpurun_out/${T}_pmc_c4 \
  lag@h:navigation:N24:B8192=gpurun_out/${T}_pmc_h_lag lag@c2:navigation:N3:B4096=gpurun_out/${T}_pmc_c2_lag \
  lag@c4:mixed:N24:B8192=gpurun_out/${T}_pmc_c4_lag \
  roll@h:navigation:N24:B8192=gpurun_out/${T}_pmc_h_roll roll@c3:navigation:N96:B1024=gpurun_out/${T}_pmc_c3_roll \
  roll@c2:navigation:N3:B4096=gpurun_out/${T}_pmc_c2_roll roll@c4:mixed:N24:B8192=gpurun_out/${T}_pmc_c4_roll > /dev/null
