# kernel-trace stats of the default bench legs on the final round-3 tree (profiles/r03k).
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r03k_prof"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$O/stats" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline > "$O/bench_under_rocprof.json" 2> "$O/rocprof.err"
rc=$?; echo "rocprof rc=$rc"; ls "$O"/stats/* | head
exit $rc
