# round 4, fourth pass: GRU w_ih precision attribution (default / fp32 dW / fp32 dh builds) on the categorical
# learner fixtures and the L = 256 value case; the narrow-critic fp32 forward; policy layer-2 and update
# residual A/B timings.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04d"; mkdir -p "$O"
worst=0
step() {
  local name=$1; shift
  "$@"; local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  [ $rc -ne 0 ] && worst=1
  return 0
}
for v in default gdw0 gdh0; do
  if [ $v = default ]; then VE=""; else VE="D2D_LIB_VARIANT=$v D2D_ALLOW_ABLATION=1"; fi
  for fx in learner_ippo_rnn_cat_ep4 learner_d2d_rnn_cat; do
    step diag_${fx}_$v env $VE timeout -k 10 120 python3 tools/gpu/gru_learner_diag.py $fx > "$O/diag_${fx}_$v.log" 2>&1
    grep "weight_ih" "$O/diag_${fx}_$v.log" | head -8
  done
  step gru_value_$v env $VE timeout -k 10 200 python3 -u -m pytest -v --timeout 180 --timeout-method thread -p no:cacheprovider -s \
    "tests/test_gru_gpu.py::test_gru_grads_long_window[f32-None-N256-L256]" > "$O/gru_value_$v.log" 2>&1
  grep -E "max\|g\|" "$O/gru_value_$v.log" | head -8
done
step critic_small timeout -k 10 300 python3 tools/gpu/critic_small.py 0 > "$O/critic_small.log" 2>&1
grep -v "^{" "$O/critic_small.log" | tail -6
step critic_tests timeout -k 10 300 python3 -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  "tests/test_learner_gpu.py::test_d2d_central_critic_split_gemm_matches_fp32" tests/test_bf16_exact_gpu.py > "$O/pytest_critic.log" 2>&1
grep -E "FAIL|passed|failed" "$O/pytest_critic.log" | tail -8
for v in default pl2f pl2f2 default pl2f2; do
  if [ $v = default ]; then VE=""; else VE="D2D_LIB_VARIANT=$v D2D_ALLOW_ABLATION=1"; fi
  step policy_$v env $VE timeout -k 10 200 python3 bench.py --legs rollout --steps 5 --warmup 2 --no-cpu-baseline \
    --rollout-steps 40 > "$O/policy_$v.json" 2> "$O/policy_$v.err"
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['rollout']; print(sys.argv[2], round(r['policy_kernel_us'],1), round(r['env_kernel_us'],1))" "$O/policy_$v.json" $v
done
step upd_ab timeout -k 10 400 python3 tools/gpu/ablate_update.py "" sub2 "" sub2 > "$O/upd_ab.json" 2>&1
cat "$O/upd_ab.json"
exit $worst
