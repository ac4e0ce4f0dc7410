# round-6 end pass (third: the final tree) on the final tree: every GPU test, smoke(), the default bench (one box).
# usage (GPU box): bash tools/gpu/run_r06z_final.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06z_final3"; mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --durations=40 --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" "$O/pytest_gpu.log" | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 2 "$O/smoke.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; tail -c 600 "$O/bench.json"
exit $rc
