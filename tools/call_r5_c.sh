# Round-5 call: C4 placement and hand-off levels, repeated: kernel time per
# placement (GSM_PLACE_XCD 1 / 0, three alternations) and PMC traffic of the
# library (XCD-local placement, three-level sums), the library with one cost
# order over the grid, and HEAD's build, twice each.
cd $GRAFT_REPO_ROOT
for rep in 1 2 3; do bash tools/gpu.sh envsweep cx$rep c4 GSM_PLACE_XCD 1 0 || exit 2; done
for rep in 1 2; do
  PMC_CONFIG=c4 PMC_SET="traffic" bash tools/pmc_quick.sh pq_c4_$rep libgsm.so ablate/head.so || exit 4
  GSM_PLACE_XCD=0 PMC_CONFIG=c4 PMC_SET="traffic" bash tools/pmc_quick.sh pq_c4x0_$rep libgsm.so || exit 4
done
