# build variants locally: bash tools/ablate.sh build "NAME:-DFLAG ..." ...
# run on GPU:             bash tools/ablate.sh run NAME ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mode=$1; shift
if [ "$mode" = build ]; then
  mkdir -p gs-marl_amd/gsmarl_amd/lib/ablate
  for spec in "$@"; do
    name=${spec%%:*}; flags=${spec#*:}
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared $flags \
      -Iinclude -Igs-marl_amd/csrc gs-marl_amd/csrc/gsm_kernels.hip gs-marl_amd/csrc/gsm_seg_kernels.hip \
      gs-marl_amd/csrc/gsm_abi.hip -o gs-marl_amd/gsmarl_amd/lib/ablate/$name.so || exit 1
    echo built $name
  done
else
  for name in "$@"; do
    GSM_LIB_PATH=gs-marl_amd/gsmarl_amd/lib/ablate/$name.so timeout -k 10 120 python tools/ablate.py || exit 1
  done
fi
