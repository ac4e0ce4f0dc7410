# round 5: the GRU gradient cases at L = 256 that the suite skips (fp32 rows and the record row-history path,
# D2D_TEST_LONG_ALL=1), once
# usage (GPU box): bash tools/gpu/run_r05y_extra.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05y"; mkdir -p "$O"
D2D_TEST_LONG_ALL=1 timeout -k 10 1000 python3 -u -m pytest tests/test_gru_gpu.py -m gpu -v \
  -k "grads_long_window and L256 and (f32 or history)" --timeout 900 --timeout-method thread -p no:cacheprovider \
  > "$O/gru_long_window_all.log" 2>&1
rc=$?; echo "gru long rc=$rc"; grep -E "passed|failed|PASSED|FAILED|SKIPPED" "$O/gru_long_window_all.log" | tail -12
exit $rc
