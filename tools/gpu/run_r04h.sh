# round 4: GRU long-window tests with the per-agent head-mask search; hidden 128 / 100 MLP kernels (policy,
# update, fused epoch); the learner traces and record tests (bitwise checks of the update kernels).
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04h"; mkdir -p "$O"
worst=0
step() {
  local name=$1; shift
  "$@"; local rc=$?
  echo "$name rc=$rc" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  [ $rc -ne 0 ] && worst=1
  return 0
}
PYT="python3 -u -m pytest -v --timeout-method thread -p no:cacheprovider -s"
step gru timeout -k 10 500 $PYT --timeout 400 tests/test_gru_gpu.py -k "long_window and None" > "$O/pytest_gru_long.log" 2>&1
grep -E "FAIL|passed|failed|ambiguous|matched|w_ih|w1:" "$O/pytest_gru_long.log" | tail -30
step h128 timeout -k 10 600 $PYT --timeout 200 tests/test_policy_gpu.py tests/test_update_gpu.py tests/test_record_gpu.py > "$O/pytest_h128.log" 2>&1
grep -E "FAIL|passed|failed" "$O/pytest_h128.log" | tail -20
exit $worst
