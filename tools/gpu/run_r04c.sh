# round 4, third pass: GRU categorical learner gradient diagnosis (default / fp32 dW / fp32 dh builds), the
# padded small-critic timing, and the tests touched since r04b.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04c"; mkdir -p "$O"
worst=0
step() {
  local name=$1; shift
  "$@"; local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  [ $rc -ne 0 ] && worst=1
  return 0
}
for fx in learner_ippo_rnn_cat_ep4 learner_d2d_rnn_cat; do
  step diag_$fx timeout -k 10 120 python3 tools/gpu/gru_learner_diag.py $fx > "$O/diag_${fx}_default.log" 2>&1
  grep -v Iteration "$O/diag_${fx}_default.log" | tail -22
  for v in gdw0 gdh0; do
    step diag_${fx}_$v env D2D_LIB_VARIANT=$v D2D_ALLOW_ABLATION=1 timeout -k 10 120 python3 tools/gpu/gru_learner_diag.py $fx > "$O/diag_${fx}_$v.log" 2>&1
    grep "policy" "$O/diag_${fx}_$v.log" | head -4
  done
done
step critic_small timeout -k 10 300 python3 tools/gpu/critic_small.py 0 > "$O/critic_small.log" 2>&1
grep -v "^{" "$O/critic_small.log" | tail -6
PYT="python3 -u -m pytest -v --timeout-method thread -p no:cacheprovider -s"
step tests timeout -k 10 500 $PYT --timeout 300 tests/test_bf16_exact_gpu.py "tests/test_gru_gpu.py::test_gru_grads_long_window" \
  "tests/test_update_gpu.py::test_fused_epoch_matches_torch_epoch" "tests/test_learner_gpu.py::test_d2d_central_critic_split_gemm_matches_fp32" \
  > "$O/pytest.log" 2>&1
grep -E "FAIL|passed|failed" "$O/pytest.log" | tail -20
exit $worst
