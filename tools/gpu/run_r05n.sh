# round 5: fused env + policy slot (tests, timing); bf16 state rows (tests, D2D iteration equality); critic forward
# prefetch A/B (PD 3 vs 2); env leg after the comb_step refactor; c5 configs leg; the c5 GRU leg with progress lines
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05n"; mkdir -p "$O"
timeout -k 10 500 python3 -u -m pytest tests/test_fused_slot_gpu.py tests/test_env_state_bf16_gpu.py -m gpu -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" "$O/pytest.log" | tail -14; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/gpu/critic_probe.py 256 > "$O/critic_probe.json" 2> "$O/critic_probe.err"
rc=$?; echo "critic rc=$rc"; cat "$O/critic_probe.json"; tail -n 3 "$O/critic_probe.err"; [ $rc -eq 0 ] || exit $rc
D2D_LIB_VARIANT=critpd2 D2D_ALLOW_ABLATION=1 timeout -k 10 300 python3 -u tools/gpu/critic_probe.py 256 > "$O/critic_probe_pd2.json" 2> "$O/critic_probe_pd2.err"
rc=$?; echo "critic pd2 rc=$rc"; cat "$O/critic_probe_pd2.json"; [ $rc -eq 0 ] || exit $rc
D2D_LIB_VARIANT=critw8 D2D_ALLOW_ABLATION=1 timeout -k 10 300 python3 -u tools/gpu/critic_probe.py 256 > "$O/critic_probe_w8.json" 2> "$O/critic_probe_w8.err"
rc=$?; echo "critic w8 rc=$rc"; cat "$O/critic_probe_w8.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u tools/gpu/fused_slot.py 65536 > "$O/fused_slot.json" 2> "$O/fused_slot.err"
rc=$?; echo "fused rc=$rc"; cat "$O/fused_slot.json"; tail -n 4 "$O/fused_slot.err"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --legs env,configs --no-cpu-baseline --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], d.get('roofline'))
c=d['configs']; print('c2', c['c2']['d2d_iteration_s'], c['c2']['phase_ms'])
[print('c5', s['agents'], s['d2d_iteration_s'], s['phase_ms']) for s in c['c5']['sweep']]" || tail -20 "$O/bench.err"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 450 python3 -u bench.py --legs gru_c5 --no-cpu-baseline --steps 5 --warmup 2 > "$O/bench_gru_c5.json" 2> "$O/bench_gru_c5.err"
rc=$?; echo "gru_c5 rc=$rc"; tail -c 1500 "$O/bench_gru_c5.json"; tail -n 8 "$O/bench_gru_c5.err"
exit $rc
