# A/B of the library against a variant build on bench configs (same box,
# alternating), plus the rollout tests of the library.
# Usage: bash tools/gpu_ab_cfg.sh TAG VARIANT CONFIG...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=$1; V=$2; shift 2; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_roll.py tests/test_gpu_roll_ragged.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_roll.log 2>&1 || { tail -40 $O/pytest_roll.log; exit 2; }
tail -1 $O/pytest_roll.log
for c in "$@"; do for rep in 1 2; do
  for lib in lib $V; do
    if [ $lib = lib ]; then L=""; else L=$PWD/gs-marl_amd/gsmarl_amd/lib/ablate/$V.so; fi
    GSM_LIB_PATH=$L timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/b_${c}_$lib.json 2>$O/b.err || { tail $O/b.err; exit 3; }
    python -c "import json;d=json.load(open('$O/b_${c}_$lib.json'));print('$c $lib', d['ms_per_step'], d['roofline']['mean_launch_us'])"
  done
done; done
