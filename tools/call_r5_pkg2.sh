# Round-5 final package, part 2: PMC passes of n12, the rollout buffer and the
# lagged chains, merged into part 1's profiles/pmc_kernels.json.
cd $GRAFT_REPO_ROOT
bash tools/gpu.sh pmc r5f n12 buffer h_lag c4_lag
