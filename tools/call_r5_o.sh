# Round-5 call: the pace target's rank offset (GSM_ROLL_PACE = q quarter
# steps; 0 = the default, equal progress; off = no pacing) re-scanned with the
# start priorities, on the driver and h lines, twice.
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  bash tools/gpu.sh envsweep pq$rep driver GSM_ROLL_PACE 0 2 4 off || exit 2
  bash tools/gpu.sh envsweep pq$rep h GSM_ROLL_PACE 0 2 4 off || exit 3
done
