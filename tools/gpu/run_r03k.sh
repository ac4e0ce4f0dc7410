# round-3 end pass on the final tree: every GPU test, smoke(), the 2-rank data-parallel rehearsal
# (VERDICT r02 item 7), the default bench and a kernel-trace stats profile of it.
# usage (GPU box): bash tools/gpu/run_r03k.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r03k_final"; mkdir -p "$O"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" "$O/pytest_gpu.log" | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$O/smoke.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29541 tools/gpu/rehearse_dp.py > "$O/rehearse_dp.log" 2>&1
rc=$?; echo "rehearse_dp rc=$rc"; grep rehearse_dp "$O/rehearse_dp.log" | cut -c1-600
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; tail -c 400 "$O/bench.json"
[ $rc -eq 0 ] || exit $rc
