# round 4, first pass: the all-agent gradient check with the relu-flip envelope and the reversed fp32
# control, the new GRU long-window and small central-critic tests (items 2, 3),
# the learner traces on the reference-gradient Adam bound, and the small-critic timing A/B.
# usage (GPU box): bash tools/gpu/run_r04a.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04a"; mkdir -p "$O"
timeout -k 10 300 python3 -u tools/gpu/ppo_grads_full_batch.py 2048 64 reversed envelope > "$O/ppo_full_2048_all_env.json" 2> "$O/ppo_full.err"
rc=$?; echo "ppo_full rc=$rc"; tail -c 1500 "$O/ppo_full_2048_all_env.json"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -s \
  tests/test_learner_gpu.py -k "matches_reference or central_critic" > "$O/pytest_learner.log" 2>&1
rc=$?; echo "pytest learner rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" "$O/pytest_learner.log" | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/gpu/critic_small.py 256 0 > "$O/critic_small.log" 2>&1
rc=$?; echo "critic_small rc=$rc"; grep -v "^{" "$O/critic_small.log" | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -s \
  tests/test_gru_gpu.py -k "long_window" > "$O/pytest_gru_long.log" 2>&1
rc=$?; echo "pytest gru rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" "$O/pytest_gru_long.log" | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -s \
  "tests/test_update_gpu.py::test_grads_on_large_rollout_vs_float64" > "$O/pytest_large.log" 2>&1
rc=$?; echo "pytest large rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed|worst|outside" "$O/pytest_large.log" | tail -30
exit $rc
