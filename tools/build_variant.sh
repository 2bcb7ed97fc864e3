# Build a diagnostic variant of libgsm.so next to the product library (never
# loaded unless GSM_LIB_PATH points at it). The sources know two flags:
# -DGSM_STAMPS (per-wave s_memtime phase stamps, read by tools/stamps*.py) and
# -DGSM_CHECKED (every rollout hand-off granule and slab address tested against
# its allocation; status 6 instead of an out-of-range access). Usage: bash tools/build_variant.sh "NAME:-DFLAG ..." ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gs-marl_amd/gsmarl_amd/lib/ablate
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  srcs=$(python -c "import __graft_entry__ as g; print(' '.join(str(g.CSRC / s) for s in g.SOURCES))")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared $flags \
    -Iinclude -Igs-marl_amd/csrc $srcs -o gs-marl_amd/gsmarl_amd/lib/ablate/$name.so || exit 1
  echo built $name
done
