# build variants locally: bash tools/ablate.sh build "NAME:-DFLAG ..." ...
# run on GPU:             bash tools/ablate.sh run NAME ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mode=$1; shift
if [ "$mode" = build ]; then
  mkdir -p gs-marl_amd/gsmarl_amd/lib/ablate
  for spec in "$@"; do
    name=${spec%%:*}; flags=${spec#*:}
    srcs=$(python -c "import __graft_entry__ as g; print(' '.join(str(g.CSRC / s) for s in g.SOURCES))")
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared $flags \
      -Iinclude -Igs-marl_amd/csrc $srcs -o gs-marl_amd/gsmarl_amd/lib/ablate/$name.so || exit 1
    echo built $name
  done
else
  for name in "$@"; do
    GSM_LIB_PATH=gs-marl_amd/gsmarl_amd/lib/ablate/$name.so timeout -k 10 120 python tools/ablate.py || exit 1
  done
fi
