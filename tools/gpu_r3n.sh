# PMC passes of the H and C4 fused rollouts + the driver's bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r3_n; mkdir -p $O
PMC_ROLL=1 bash tools/pmc.sh r3_n/pmc_h_roll --config h > $O/pmc_h.log 2>&1 || { tail $O/pmc_h.log; exit 2; }
PMC_ROLL=1 bash tools/pmc.sh r3_n/pmc_c4_roll --config c4 > $O/pmc_c4.log 2>&1 || { tail $O/pmc_c4.log; exit 3; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 4; }
python -c "import json;d=json.load(open('$O/bench_driver.json'));r=d['roofline'];print('driver', d['value'], d['ms_per_step'], r['mean_launch_us'])"
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_h.json 2> $O/bench_h.err || { tail -20 $O/bench_h.err; exit 5; }
python -c "import json;d=json.load(open('$O/bench_h.json'));r=d['roofline'];print('h', d['value'], d['ms_per_step'], r['mean_launch_us'])"
