# round 5: actor dZ-once, deferred iPPO values (actor-only rollout slot), the fused D2D central critic:
# timing + tests + the rollout / ppo / train / configs bench legs
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05h"; mkdir -p "$O"
timeout -k 10 200 python3 -u tools/gpu/upd_ab.py 2048 64 > "$O/upd_ab_h64.json" 2>> "$O/upd_ab.err"
rc=$?; echo "upd_ab rc=$rc"; cat "$O/upd_ab_h64.json"; [ $rc -eq 0 ] || { tail -20 "$O/upd_ab.err"; exit $rc; }
timeout -k 10 800 python3 -u -m pytest tests/test_record_gpu.py tests/test_update_gpu.py tests/test_policy_gpu.py \
  tests/test_learner_gpu.py tests/test_drivers_gpu.py tests/test_data_parallel_gpu.py -m gpu -v -k "not 8192" --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" "$O/pytest.log" | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u bench.py --legs rollout,ppo,train,configs --no-cpu-baseline --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
r=d['rollout']; print('slot', r['policy_kernel_us'], r['env_kernel_us'], r['values']); p=d['ppo']; print('ppo', p['updates_per_s'], p['kernels']['actor']['ms'], p['kernels']['critic']['ms'])
t=d['train']; print('train', t['s_per_iteration'], t['phase_ms'])
c=d['configs']; print('c2', c['c2']['d2d_iteration_s'], c['c2']['phase_ms'])
[print('c5', s['agents'], s['d2d_iteration_s'], s['phase_ms']) for s in c['c5']['sweep']]" || tail -20 "$O/bench.err"
exit $rc
