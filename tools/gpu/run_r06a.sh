# round 6, first pass: the new / changed GPU tests (bench self-launch, deferred values at H 64 / 128, ragged-H
# central critic) and the default bench on this round's starting tree.
# usage (GPU box): bash tools/gpu/run_r06a.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06a"; mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests/test_bench_launch_gpu.py tests/test_update_gpu.py::test_deferred_values_equal_rollout_values \
  tests/test_learner_gpu.py::test_d2d_central_critic_split_gemm_matches_fp32 -m gpu -v --timeout 450 --timeout-method thread \
  -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" "$O/pytest_gpu.log" | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; tail -c 600 "$O/bench.json"
exit $rc
