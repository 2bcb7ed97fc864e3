# Same-box bench lines (default and the driver's 20-step) of the library and
# of variant builds (lib/ablate/NAME.so via GSM_LIB_PATH), alternated twice,
# then the launch probe of the library. Usage: bash tools/gpu_bench_ab.sh TAG variant...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; shift; mkdir -p $O
for rep in 1 2; do
  for v in lib "$@"; do
    if [ "$v" = lib ]; then L=""; else L=gs-marl_amd/gsmarl_amd/lib/ablate/$v.so; fi
    GSM_LIB_PATH=$L timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/drv_${v}_$rep.json 2> $O/drv_${v}_$rep.err || exit 4
    GSM_LIB_PATH=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/h_${v}_$rep.json 2> $O/h_${v}_$rep.err || exit 4
    python -c "import json; d=json.load(open('$O/drv_${v}_$rep.json')); e=json.load(open('$O/h_${v}_$rep.json')); print('$v', 'driver', d['ms_per_step'], 'h', e['ms_per_step'], e['roofline']['mean_launch_us'])"
  done
done
timeout -k 10 120 python tools/probe_launch.py > $O/probe_lib.json && cat $O/probe_lib.json
