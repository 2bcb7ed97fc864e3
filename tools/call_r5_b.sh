# Round-5 call: launch-timeline stamps of a 20-step graph (plain, and across an
# episode boundary) and the granule memory A/B (uncached vs hipMalloc).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/st1
S=$GRAFT_REPO_ROOT/gs-marl_amd/gsmarl_amd/lib/ablate/stamps.so
GSM_LIB_PATH=$S STAMPS_NPZ=gpurun_out/st1/h20.npz timeout -k 10 200 python3 tools/stamps_h_timeline.py > gpurun_out/st1/h20.json 2> gpurun_out/st1/h20.err || exit 1
GSM_LIB_PATH=$S ROLL_START=90 STAMPS_NPZ=gpurun_out/st1/h20b.npz timeout -k 10 200 python3 tools/stamps_h_timeline.py > gpurun_out/st1/h20b.json 2> gpurun_out/st1/h20b.err || exit 1
for rep in 1 2; do
  for l in driver h c2; do
    bash tools/gpu.sh envsweep gran$rep $l GSM_GRAN_MEM uc hip || exit 2
  done
done
