# round 5: the GRU policy kernel's padding table in global memory for history_len > 64 (xp_n_agents' GRU learner):
# GRU + learner tests, then the c5 GRU leg and the xp_load GRU leg
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05zf"; mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest tests/test_gru_gpu.py tests/test_learner_gpu.py -m gpu -q -x \
  --timeout 400 --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --legs gru,gru_c5 --steps 5 --warmup 2 --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
g=d['gru']; print('gru', g['policy_slot']['ms'], g['update']['ms'], g['d2d_iteration_s']); print(d['c5_gru_summary'])"
exit $rc
