# round 6: the D2DEnv compact record (single_kernel, ABI 14): D2DEnv tests, learner traces on the D2DEnv (now on the
# record), the record / baselines / drivers suites, then the d2denv bench leg (fp32 rows and record).
# usage (GPU box): bash tools/gpu/run_r06f.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06f"; mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest tests/test_d2denv_gpu.py tests/test_learner_gpu.py tests/test_record_gpu.py tests/test_baselines_gpu.py \
  tests/test_drivers_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" "$O/pytest_gpu.log" | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --legs d2denv --steps 5 --warmup 2 --no-cpu-baseline > "$O/bench_d2denv.json" 2> "$O/bench_d2denv.err"
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; s=open('$O/bench_d2denv.json').read(); d=json.loads(s[s.index('{\"metric\"'):])['d2denv']; r=d.pop('record'); print(json.dumps(d)); print(json.dumps(r))"
exit $rc
