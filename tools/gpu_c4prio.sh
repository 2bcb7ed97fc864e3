# A/B: C4 bench line with the base build vs the cold-solve priority build, alternated
# (variants from tools/ablate.sh build "base:" "coldprio:-DGSM_COLD_PRIO", before the
# raised priority became unconditional in gsm_ragged_kernels.hip).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/c4prio; mkdir -p $O
for rep in 1 2; do for v in base coldprio; do
GSM_LIB_PATH=gs-marl_amd/gsmarl_amd/lib/ablate/$v.so timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { tail -20 $O/${v}_$rep.err; exit 5; }
python -c "import json; d=json.load(open('$O/${v}_$rep.json')); print('$v', $rep, d['ms_per_step'], d['roofline']['mean_launch_us'])"
done; done
