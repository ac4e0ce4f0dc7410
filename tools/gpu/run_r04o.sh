# round 4: forced policy launches at one resident round (forced bytes through the DMA ring) -- tests, c2/c5 timing
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04o"; mkdir -p "$O"
timeout -k 10 700 python3 -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_policy_gpu.py tests/test_learner_gpu.py tests/test_record_gpu.py tests/test_drivers_gpu.py tests/test_update_gpu.py > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed" "$O/pytest.log" | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --legs configs --steps 5 --warmup 2 --no-cpu-baseline > "$O/configs.json" 2> "$O/configs.err"
rc=$?; echo "configs rc=$rc"
grep "^{" "$O/configs.json" | python3 -c "
import json,sys
c=json.loads(sys.stdin.read())['configs']
print('c2', round(c['c2']['d2d_iteration_s']*1e3,2), {k: round(v,2) for k,v in c['c2']['phase_ms'].items()})
for s in c['c5']['sweep']: print('c5', s['agents'], round(s['d2d_iteration_s']*1e3,2), {k: round(v,2) for k,v in s['phase_ms'].items()})"
exit $rc
