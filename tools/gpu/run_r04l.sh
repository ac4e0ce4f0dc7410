# round 4: central critic on the three-way dPre split -- learner traces (hidden-128 D2D) and the small-critic timing
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04l"; mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider -s \
  tests/test_learner_gpu.py tests/test_bf16_exact_gpu.py > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed" "$O/pytest.log" | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/gpu/critic_small.py > "$O/critic_small.log" 2>&1
rc=$?; echo "critic_small rc=$rc"; cat "$O/critic_small.log" | grep -v amdgpu.ids
exit $rc
