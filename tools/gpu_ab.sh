# Same-box A/B of the library and variant builds with tools/probe_launch.py,
# alternated. Usage: bash tools/gpu_ab.sh TAG variant...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; shift; mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 120 python tools/probe_launch.py > $O/lib_$rep.json || exit 3
  python -c "import json;d=json.load(open('$O/lib_$rep.json'));print('lib', d['roll20_us'], d['roll20_b2b_us'], d['roll100_events_us_per_step'], d['roll100_b2b_us_per_step'], d['gave_up'])"
  for v in "$@"; do
    GSM_LIB_PATH=gs-marl_amd/gsmarl_amd/lib/ablate/$v.so timeout -k 10 120 python tools/probe_launch.py > $O/${v}_$rep.json || exit 3
    python -c "import json;d=json.load(open('$O/${v}_$rep.json'));print('$v', d['roll20_us'], d['roll20_b2b_us'], d['roll100_events_us_per_step'], d['roll100_b2b_us_per_step'], d['gave_up'])"
  done
done
