# round 4: the learner traces incl. the hidden-128 reference fixtures, and the policy tests (Philox default back)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04k"; mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider -s \
  tests/test_learner_gpu.py tests/test_policy_gpu.py > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed|first-step" "$O/pytest.log" | tail -25
exit $rc
