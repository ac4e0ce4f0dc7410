# round 4, fifth pass: the whole GPU suite on the tree with the GRU fixes (fractional-x dW_ih, 64-step
# accumulation chains) and the sub2 residuals, the GRU categorical learner diagnosis after the fix, and the
# 2-rank product rehearsal at the benched 64 agents x 8 channels.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04e"; mkdir -p "$O"
worst=0
step() {
  local name=$1; shift
  "$@"; local rc=$?
  echo "$name rc=$rc" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  [ $rc -ne 0 ] && worst=1
  return 0
}
step pytest timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$O/pytest_gpu.log" 2>&1
grep -E "FAIL|passed|failed" "$O/pytest_gpu.log" | tail -25
for fx in learner_ippo_rnn_cat_ep4 learner_d2d_rnn_cat; do
  step diag_$fx timeout -k 10 120 python3 tools/gpu/gru_learner_diag.py $fx > "$O/diag_$fx.log" 2>&1
  grep "weight_ih" "$O/diag_$fx.log" | head -4
done
step rehearse env D2D_REHEARSE_N=64 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29541 tools/gpu/rehearse_dp.py > "$O/rehearse_dp_n64.log" 2>&1
grep rehearse_dp "$O/rehearse_dp_n64.log" | cut -c1-1500
exit $worst
