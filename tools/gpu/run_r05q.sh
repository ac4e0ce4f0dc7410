# round 5: the critic forward with W1 image slices two iterations ahead (D2D_CRITIC_WPD=2, on the XLDS path): central-critic
# tests, probe A/B against W1 slices one iteration ahead (critwpd1), the configs leg
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05q"; mkdir -p "$O"
timeout -k 10 400 python3 -u -m pytest tests/test_learner_gpu.py tests/test_env_state_bf16_gpu.py -m gpu -v -k "central_critic or d2d_iteration" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" "$O/pytest.log" | tail -8; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 300 python3 -u tools/gpu/critic_probe.py 256 > "$O/critic_probe_xl_$k.json" 2> "$O/critic_probe_xl_$k.err" || exit 11
  D2D_LIB_VARIANT=critwpd1 D2D_ALLOW_ABLATION=1 timeout -k 10 300 python3 -u tools/gpu/critic_probe.py 256 > "$O/critic_probe_wpd1_$k.json" 2> "$O/critic_probe_wpd1_$k.err" || exit 12
  python3 -c "
import json
for n in ('xl', 'wpd1'):
    d = json.loads(open('$O/critic_probe_' + n + '_$k.json').read())
    print(n, $k, 'fwd', round(d['fwd_ms'], 3), 'dw1', round(d['dw1_ms'], 3))"
done
timeout -k 10 400 python3 -u bench.py --legs configs --no-cpu-baseline --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
c=d['configs']; print('c2', c['c2']['d2d_iteration_s'], c['c2']['phase_ms'])
[print('c5', s['agents'], s['d2d_iteration_s'], s['phase_ms']) for s in c['c5']['sweep']]" || tail -20 "$O/bench.err"
exit $rc
