# round 6: carried GRU state (tests + c5 GRU leg), the fused slot's oracle pin, the D2DEnv kernel's PMC traffic.
# usage (GPU box): bash tools/gpu/run_r06b.sh <commit>
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06b"; mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests/test_gru_gpu.py tests/test_fused_slot_gpu.py -k "carr or fused_slot" -m gpu -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" "$O/pytest_gpu.log" | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --legs gru,gru_c5 --steps 5 --warmup 2 --no-cpu-baseline > "$O/bench_gru.json" 2> "$O/bench_gru.err"
rc=$?; echo "bench rc=$rc"; tail -c 400 "$O/bench_gru.json"
[ $rc -eq 0 ] || exit $rc
bash tools/gpu/profile_single.sh r06b "$1"
rc=$?; echo "profile rc=$rc"; cat "$R/gpurun_out/prof_r06b/pmc_traffic_single.json"
exit $rc
