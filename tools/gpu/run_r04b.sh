# round 4, second pass: learner traces on the reference-gradient bound, the small-critic timing A/B,
# the GRU long-window tests, the all-agent headline-batch gradient test, the dot2 special-input probe.
# A step that fails its assertions (rc 1) does not stop the pass; a timeout / abort / fault does.
# usage (GPU box): bash tools/gpu/run_r04b.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04b"; mkdir -p "$O"
worst=0
step() {  # name, then the command; stops the pass on anything but pass / assertion failure
  local name=$1; shift
  "$@"; local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  [ $rc -ne 0 ] && worst=1
  return 0
}
PYT="python3 -u -m pytest -v --timeout-method thread -p no:cacheprovider -s"
step learner timeout -k 10 400 $PYT --timeout 200 tests/test_learner_gpu.py > "$O/pytest_learner.log" 2>&1
grep -E "FAIL|passed|failed|first-step" "$O/pytest_learner.log" | tail -30
step critic_small timeout -k 10 300 python3 tools/gpu/critic_small.py 256 0 > "$O/critic_small.log" 2>&1
grep -v "^{" "$O/critic_small.log" | tail -12
step gru_long timeout -k 10 600 $PYT -x --timeout 300 tests/test_gru_gpu.py -k "long_window" > "$O/pytest_gru_long.log" 2>&1
grep -E "PASS|FAIL|passed|failed" "$O/pytest_gru_long.log" | tail -30
step large timeout -k 10 300 $PYT --timeout 280 "tests/test_update_gpu.py::test_grads_on_large_rollout_vs_float64" > "$O/pytest_large.log" 2>&1
grep -E "PASS|FAIL|passed|failed|worst|outside" "$O/pytest_large.log" | tail -20
step probe timeout -k 10 60 tools/gpu/probe/dot2_probe > "$O/dot2_probe.txt" 2>&1
tail -25 "$O/dot2_probe.txt"
exit $worst
