# round 5: the fused env + policy slot prototype (bit-exactness tests, slot timing at 65,536 envs, whole rollouts);
# the env leg after the comb_step refactor; the c5 GRU leg with progress lines
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05m"; mkdir -p "$O"
timeout -k 10 400 python3 -u -m pytest tests/test_fused_slot_gpu.py -m gpu -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" "$O/pytest.log" | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u tools/gpu/fused_slot.py 65536 > "$O/fused_slot.json" 2> "$O/fused_slot.err"
rc=$?; echo "fused rc=$rc"; cat "$O/fused_slot.json"; tail -n 4 "$O/fused_slot.err"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u bench.py --legs env --no-cpu-baseline --steps 20 --warmup 5 > "$O/bench_env.json" 2> "$O/bench_env.err"
rc=$?; echo "env rc=$rc"; tail -c 800 "$O/bench_env.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/gpu/critic_probe.py 256 > "$O/critic_probe.json" 2> "$O/critic_probe.err"
rc=$?; echo "critic rc=$rc"; cat "$O/critic_probe.json"; tail -n 3 "$O/critic_probe.err"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 450 python3 -u bench.py --legs gru_c5 --no-cpu-baseline --steps 5 --warmup 2 > "$O/bench_gru_c5.json" 2> "$O/bench_gru_c5.err"
rc=$?; echo "gru_c5 rc=$rc"; tail -c 1500 "$O/bench_gru_c5.json"; tail -n 8 "$O/bench_gru_c5.err"
exit $rc
