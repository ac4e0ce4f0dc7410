# round-5 end: the default bench once more after the PMC restamp (its legs read profiles/pmc_*.json)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05z_bench"; mkdir -p "$O"
timeout -k 10 400 python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; tail -c 400 "$O/bench.json"
exit $rc
