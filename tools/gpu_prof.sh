# rocprofv3 kernel stats of the default bench command and of C4 (profiles/<tag>_kernel_stats_*.csv).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${1:-r2_n}; mkdir -p $O
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_h" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/$O/prof_h.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/$O/prof_h.log"; exit 6; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_c4" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config c4 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$O/prof_c4.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/$O/prof_c4.log"; exit 7; }
find "$GRAFT_REPO_ROOT/$O" -name "*kernel_stats.csv"
