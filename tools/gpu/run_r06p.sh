# round 6: D2D-PPO's epoch-start forced log-prob pass with the actions agent-major (forced_layout 1, ABI 15) and
# actions = NULL: probe timings, the policy / record / GRU-forced / learner tests, and the configs leg (c2, c5 sweep).
# usage (GPU box): bash tools/gpu/run_r06p.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06p"; mkdir -p "$O"
for k in 1 2; do
  timeout -k 10 240 python3 -u tools/gpu/policy_mode_probe.py > "$O/probe_$k.json" 2> "$O/probe_$k.err" || exit 11
  cat "$O/probe_$k.json"
done
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_policy_gpu.py \
  tests/test_record_gpu.py tests/test_learner_gpu.py tests/test_update_gpu.py -k "not large_rollout" > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit 12
timeout -k 10 600 python3 -u bench.py --legs configs --steps 5 --warmup 2 --no-cpu-baseline > "$O/bench_configs.json" 2> "$O/bench_configs.err"
echo "bench rc=$?"
python3 - "$O/bench_configs.json" <<'PY'
import json, sys
s = open(sys.argv[1]).read(); d = json.loads(s[s.index('{"metric"'):])
c = d["configs"]
print("c2", round(c["c2"]["d2d_iteration_s"] * 1e3, 2), {k: round(v, 2) for k, v in c["c2"]["phase_ms"].items()})
for r in c["c5"]["sweep"]:
    print("c5", r["agents"], round(r["d2d_iteration_s"] * 1e3, 2), {k: round(v, 2) for k, v in r["phase_ms"].items()})
PY
