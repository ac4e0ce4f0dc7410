# round 4 end: the 2-rank product-path rehearsal (gloo on one GPU) at the benched 64 agents x 8 channels, final tree
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04t"; mkdir -p "$O"
D2D_REHEARSE_N=64 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29541 tools/gpu/rehearse_dp.py > "$O/rehearse_dp_n64.log" 2>&1
rc=$?; echo "rehearse rc=$rc"; grep -o '"violations.*' "$O/rehearse_dp_n64.log"

[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/gpu/upd_concurrency_probe.py > "$O/upd_conc.json" 2> "$O/upd_conc.err"
rc=$?; echo "conc rc=$rc"; cat "$O/upd_conc.json"; [ $rc -eq 0 ] || tail -3 "$O/upd_conc.err"
exit $rc
