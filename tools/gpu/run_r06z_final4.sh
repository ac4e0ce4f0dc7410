# round-6 end pass (fourth: the final tree, four-wave A = 8 policy kernels): every GPU test, smoke(), the default bench,
# then the rollout leg's policy-kernel counters (the kernel changed after the b12ff77 re-stamp).  SKIP_TESTS=1 skips the
# test step (already run on this build).
# usage (GPU box): bash tools/gpu/run_r06z_final4.sh <commit>
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06z_final4"; mkdir -p "$O"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --durations=40 --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$O/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" "$O/pytest_gpu.log" | tail -3
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 2 "$O/smoke.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; tail -c 300 "$O/bench.json"
[ $rc -eq 0 ] || exit $rc
if [ "${SKIP_PMC:-0}" != 1 ]; then
  bash "$R/tools/gpu/pmc_legs.sh" r06f "$1" rollout > "$O/pmc_rollout.log" 2>&1
  rc=$?; echo "pmc rollout rc=$rc"; tail -n 2 "$O/pmc_rollout.log"
  cp "$R/gpurun_out/pmcl_r06f/pmc_mfma_rollout.json" "$O/" 2>/dev/null
  cp "$(ls "$R"/gpurun_out/pmcl_r06f/rollout/stats/*kernel_stats.csv | head -1)" "$O/rollout_kernel_stats.csv" 2>/dev/null
  rm -rf "$R/gpurun_out/pmcl_r06f"
fi
exit $rc
