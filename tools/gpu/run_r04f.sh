# round 4: long-window GRU value diagnosis and the 64-agent 2-rank rehearsal (scratch outside gpurun_out).
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04f"; mkdir -p "$O"
timeout -k 10 400 python3 -u tools/gpu/gru_long_diag.py > "$O/gru_long_diag.log" 2>&1
rc=$?; echo "diag rc=$rc"; grep -v Warn "$O/gru_long_diag.log" | grep -E "^(value|sigmoid)|^   " | cut -c1-900
[ $rc -eq 0 ] || exit $rc
D2D_REHEARSE_N=64 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29541 tools/gpu/rehearse_dp.py > "$O/rehearse_dp_n64.log" 2>&1
rc=$?; echo "rehearse rc=$rc"; grep -o '"violations.*' "$O/rehearse_dp_n64.log"
exit $rc
