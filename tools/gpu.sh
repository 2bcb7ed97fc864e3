# The one GPU measurement script (run on the box through gpurun). Every step
# has its own time limit; the first failure ends the call.
#
#   bash tools/gpu.sh tests TAG [pytest -k expr]   GPU tests + smoke
#   bash tools/gpu.sh lines TAG [line ...]         bench lines (default: all)
#        line: h driver c2 c3 c4 n6 n12 eager policy policyg policygc policyg10 policygc10 buffer vecenv_c2 vecenv_h
#   bash tools/gpu.sh pmc TAG [which ...]          PMC passes -> profiles/pmc_kernels.json
#        which: h c2 c3 c4 n6 n12 buffer (rollouts), h_step c4_step h_lag c4_lag
#   bash tools/gpu.sh prof TAG [line ...]          rocprofv3 --kernel-trace --stats of bench lines
#   bash tools/gpu.sh package TAG                  pmc (all) + tests + lines (all) + prof (h c4 eager policy buffer)
#   bash tools/gpu.sh ab TAG variant ...           same-box A/B: bench lines h / driver / c4 (AB_LINES) of the
#        library and of lib/ablate/VARIANT.so builds (tools/build_variant.sh), alternated twice
#   bash tools/gpu.sh envsweep TAG LINE VAR v1 v2 ...   one bench line under VAR=v (e.g. GSM_ROLL_DEPTH)
#   bash tools/gpu.sh stamps TAG which ...         phase stamps of the lib/ablate/stamps.so build
#        which: h (launch timeline) c2 c3 c4 (tools/stamps_*.py)
# Outputs under gpurun_out/TAG/ (copy what is judged into profiles/).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
CMD=$1; T=$2; shift 2
O=gpurun_out/$T
mkdir -p $O

# bench arguments of a named line
line_args() {
  case $1 in
    h) echo "" ;;
    driver) echo "--gpus 1 --steps 20 --warmup 5" ;;
    c2|c3|c4) echo "--config $1 --cpu-seconds 10" ;;
    n6) echo "--n-agents 6 --no-cpu-baseline" ;;
    n12) echo "--n-agents 12 --no-cpu-baseline" ;;
    eager) echo "--eager --steps 200 --warmup 20 --no-cpu-baseline" ;;
    policy) echo "--policy --steps 200 --warmup 20 --no-cpu-baseline" ;;
    policyg) echo "--policy-graph --steps 200 --warmup 20 --no-cpu-baseline" ;;
    policygc) echo "--policy-graph --policy-act cont --steps 200 --warmup 20 --no-cpu-baseline" ;;
    policygc10) echo "--policy-graph --policy-graph-steps 10 --policy-act cont --steps 200 --warmup 20 --no-cpu-baseline" ;;
    policyg10) echo "--policy-graph --policy-graph-steps 10 --steps 200 --warmup 20 --no-cpu-baseline" ;;
    buffer) echo "--buffer --no-cpu-baseline" ;;
    vecenv_c2) echo "--config c2 --vec-env numpy-dense --steps 200 --warmup 20 --no-cpu-baseline" ;;
    vecenv_h) echo "--vec-env numpy-coo --steps 100 --warmup 10 --no-cpu-baseline" ;;
    *) echo "unknown line $1" >&2; return 1 ;;
  esac
}
show() {   # one summary row of a bench line
  python - "$1" "$2" <<'EOF'
import json, sys
d = json.load(open(sys.argv[2])); r = d.get("roofline") or {}
print(sys.argv[1], d["value"], d["ms_per_step"], "bound", r.get("bound"), r.get("binding_pipe"), "frac", r.get("frac"),
      "phys", r.get("hbm_frac_physical"), "valu", r.get("valu_frac"), "salu", r.get("salu_frac"),
      "launch_us", r.get("mean_launch_us"), "pmc", (r.get("pmc") or {}).get("status"))
EOF
}
run_line() {   # NAME [env assignments via the caller]
  local a; a=$(line_args $1) || exit 9
  timeout -k 10 300 python3 bench.py $a > $O/bench_$1.json 2> $O/bench_$1.err || { tail -20 $O/bench_$1.err; exit 5; }
  show $1 $O/bench_$1.json
}
pmc_one() {   # WHICH: PMC passes (tools/pmc.sh) of one configuration
  local w=$1 env="" args=""
  case $w in
    h|c2|c3|c4) env="PMC_ROLL=1"; args="--config $w" ;;
    n6|n12) env="PMC_ROLL=1"; args="--n-agents ${w#n}" ;;
    buffer) env="PMC_ROLL=1"; args="--buffer" ;;
    h_step|c4_step) args="--config ${w%_step}" ;;
    h_lag|c4_lag) env="PMC_GRAPH=1"; args="--config ${w%_lag}" ;;
    *) echo "unknown pmc $w"; exit 9 ;;
  esac
  env $env timeout -k 10 400 bash tools/pmc.sh ${T}_pmc_$w $args > $O/pmc_$w.log 2>&1 || { tail -20 $O/pmc_$w.log; exit 1; }
  mkdir -p $O/pmc/$w && cp gpurun_out/${T}_pmc_$w/summary.txt $O/pmc/$w/
}
pmc_key() {   # the profiles/pmc_kernels.json key spec of a collected configuration
  case $1 in
    h) echo "roll@h:navigation:N24:B8192" ;;
    c2) echo "roll@c2:navigation:N3:B4096" ;;
    c3) echo "roll@c3:navigation:N96:B1024" ;;
    c4) echo "roll@c4:mixed:N24:B8192" ;;
    n6) echo "roll@h:navigation:N6:B8192" ;;
    n12) echo "roll@h:navigation:N12:B8192" ;;
    buffer) echo "roll>rollbuf@b:navigation:N24:B8192" ;;
    h_step) echo "step+emit@h:navigation:N24:B8192" ;;
    c4_step) echo "step+emit@c4:mixed:N24:B8192" ;;
    h_lag) echo "lag@h:navigation:N24:B8192" ;;
    c4_lag) echo "lag@c4:mixed:N24:B8192" ;;
  esac
}

case $CMD in
  tests)
    K=(); [ -n "$1" ] && K=(-k "$1")
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider "${K[@]}" > $O/pytest_gpu.log 2>&1; rc=$?
    grep -E "passed|failed|error" $O/pytest_gpu.log | tail -3
    [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_gpu.log | head -80; exit $rc; }
    grep "max |" $O/pytest_gpu.log | sort -k2 | tail -2
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
    tail -1 $O/smoke.log ;;
  lines)
    for l in ${@:-h driver c2 c3 c4 n6 n12 eager policy policyg policygc policyg10 policygc10 buffer vecenv_c2 vecenv_h}; do run_line $l; done ;;
  pmc)
    specs=""
    for w in ${@:-h c2 c3 c4 n6 n12 buffer h_lag c4_lag}; do pmc_one $w; specs="$specs $(pmc_key $w)=gpurun_out/${T}_pmc_$w"; done
    python tools/pmc_traffic.py profiles/pmc_kernels.json $specs > /dev/null || exit 1
    mkdir -p gpurun_out/profiles_new && cp profiles/pmc_kernels.json gpurun_out/profiles_new/ && cp profiles/pmc_kernels.json $O/pmc/
    echo "pmc collected: $specs" ;;
  prof)
    for l in ${@:-h c4}; do
      a=$(line_args $l) || exit 9
      ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_$l" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $a --no-cpu-baseline > "$GRAFT_REPO_ROOT/$O/prof_$l.log" 2>&1 ) || { tail -20 $O/prof_$l.log; exit 6; }
      f=$(ls $O/prof_$l/*kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && head -4 "$f"
    done ;;
  package)
    rm -f profiles/pmc_kernels.json
    bash tools/gpu.sh pmc $T || exit 1
    bash tools/gpu.sh tests $T || exit 2
    bash tools/gpu.sh lines $T || exit 4
    bash tools/gpu.sh prof $T h c4 c2 eager policygc buffer || exit 6 ;;
  ab)
    for rep in 1 2; do
      for v in lib "$@"; do
        L=""; [ "$v" = lib ] || L=gs-marl_amd/gsmarl_amd/lib/ablate/$v.so
        for l in ${AB_LINES:-driver h c4}; do
          a=$(line_args $l) || exit 9
          GSM_LIB_PATH=$L timeout -k 10 300 python3 bench.py $a --no-cpu-baseline > $O/${l}_${v}_$rep.json 2> $O/${l}_${v}_$rep.err || { tail -20 $O/${l}_${v}_$rep.err; exit 4; }
          show "$v/$l/$rep" $O/${l}_${v}_$rep.json
        done
      done
    done ;;
  envsweep)
    l=$1; var=$2; shift 2
    a=$(line_args $l) || exit 9
    for v in "$@"; do
      env $var=$v timeout -k 10 300 python3 bench.py $a --no-cpu-baseline > $O/${l}_$v.json 2> $O/${l}_$v.err || { tail -20 $O/${l}_$v.err; exit 4; }
      show "$var=$v" $O/${l}_$v.json
    done ;;
  stamps)
    for w in "$@"; do
      case $w in h) sc=tools/stamps_h_timeline.py ;; c2|c3|c4) sc=tools/stamps_${w}_roll.py ;; *) echo "unknown stamps $w"; exit 9 ;; esac
      GSM_LIB_PATH=gs-marl_amd/gsmarl_amd/lib/ablate/stamps.so timeout -k 10 200 python3 $sc > $O/stamps_$w.json 2> $O/stamps_$w.err || { tail -20 $O/stamps_$w.err; exit 7; }
      cat $O/stamps_$w.json
    done ;;
  *) echo "unknown command $CMD"; exit 9 ;;
esac
