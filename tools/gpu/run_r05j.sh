# round 5: central-critic test against float64 (flip-aware bar), incl. the hipBLASLt path at H = 128
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05j"; mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests/test_learner_gpu.py -m gpu -v -s -k "central_critic" --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|: linear1" "$O/pytest.log" | tail -30
exit $rc
