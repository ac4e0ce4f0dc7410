# round 5: small env batches spread over every CU (run_env block sizing): the env tests (bit-exact against the oracle
# and the reference traces at every shape), the configs leg (c2 / c5 env-step rates and iterations)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05s"; mkdir -p "$O"
timeout -k 10 500 python3 -u -m pytest tests/test_env_gpu.py tests/test_d2denv_gpu.py tests/test_record_gpu.py -m gpu -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --legs configs --no-cpu-baseline --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
c=d['configs']; print('c2', c['c2']['env_steps_per_s'], c['c2']['env_kernel']['kernel_avg_us'], c['c2']['env_kernel']['step_us'], c['c2']['d2d_iteration_s'])
[print('c5', s['agents'], s['env_steps_per_s'], s['env_kernel']['kernel_avg_us'], s['env_kernel']['step_us'], s['d2d_iteration_s'], s['phase_ms']['rollout']) for s in c['c5']['sweep']]" || tail -20 "$O/bench.err"
exit $rc
