# Segmented-path iteration: the full GPU test suite, then ablate.py timings of
# the headline (H) and C2 step / lagged-step / emit kernels with the in-tree
# library. Usage: bash tools/gpu_seg.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-seg}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest_gpu.log | head -60; exit $rc; }
timeout -k 10 120 python tools/ablate.py > $O/abl_h.json 2>&1 || { tail -5 $O/abl_h.json; exit 3; }
cat $O/abl_h.json
ABL_N=3 ABL_B=4096 timeout -k 10 120 python tools/ablate.py > $O/abl_c2.json 2>&1 || { tail -5 $O/abl_c2.json; exit 4; }
cat $O/abl_c2.json
