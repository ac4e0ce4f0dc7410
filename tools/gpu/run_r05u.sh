# round 5: critic_t at 2 waves per SIMD by default: update / record / learner tests, real-rollout timing, train leg
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05u"; mkdir -p "$O"
timeout -k 10 700 python3 -u -m pytest tests/test_update_gpu.py tests/test_record_gpu.py tests/test_learner_gpu.py -m gpu -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/gpu/upd_ab.py 2048 64 10 real > "$O/upd_ab_real.json" 2> "$O/upd_ab_real.err" || exit 11
cat "$O/upd_ab_real.json"
timeout -k 10 500 python3 -u bench.py --legs ppo,train --no-cpu-baseline --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('ppo', d['ppo_updates_per_s'], d['ppo']['actor']['ms'], d['ppo']['critic']['ms']); print('train', d['train_s_per_iteration'], d['train_phase_ms'])" || tail -20 "$O/bench.err"
exit $rc
