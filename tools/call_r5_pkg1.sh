# Round-5 final package, part 1: PMC passes of the rollouts h c2 c3 c4 n6
# (profiles/pmc_kernels.json re-collected on this code object).
cd $GRAFT_REPO_ROOT
rm -f profiles/pmc_kernels.json
bash tools/gpu.sh pmc r5f h c2 c3 c4 n6
