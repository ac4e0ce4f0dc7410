# round 5: the fused central critic at H = 128 (diagnostic) and the D2D learner tests after the operand-padding fix
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05i"; mkdir -p "$O"
for cfg in "128 3848 1280" "64 3848 1280" "128 256 1280" "128 3848 256"; do
  timeout -k 10 120 python3 -u tools/gpu/critic_diag.py $cfg >> "$O/critic_diag.json" 2>> "$O/critic_diag.err" || { tail -5 "$O/critic_diag.err"; exit 3; }
done
cat "$O/critic_diag.json"
timeout -k 10 600 python3 -u -m pytest tests/test_learner_gpu.py -m gpu -v -s -k "d2d" --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|: linear1" "$O/pytest.log" | tail -30
exit $rc
