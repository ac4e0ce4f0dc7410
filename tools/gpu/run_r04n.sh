# round 4: one-round policy launches -- policy / learner / driver / record tests and the rollout leg
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04n"; mkdir -p "$O"
timeout -k 10 700 python3 -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_policy_gpu.py tests/test_learner_gpu.py tests/test_record_gpu.py tests/test_drivers_gpu.py > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed" "$O/pytest.log" | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench.py --legs rollout --steps 5 --warmup 2 --no-cpu-baseline --rollout-steps 60 > "$O/rollout.json" 2> "$O/rollout.err"
rc=$?; echo "rollout rc=$rc"; grep "^{" "$O/rollout.json" | python3 -c "
import json,sys
r=json.loads(sys.stdin.read())['rollout']; print({k: r[k] for k in ('policy_kernel_us','env_kernel_us','env_steps_per_s')})"
exit $rc
