# round 6: the A = 8 policy instantiations at four waves per SIMD (D2D_POLICY_AF8_WAVES): probe, the policy / record /
# learner tests, and the configs leg.
# usage (GPU box): bash tools/gpu/run_r06x.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06x"; mkdir -p "$O"
timeout -k 10 240 python3 -u tools/gpu/policy_mode_probe.py > "$O/probe.json" 2> "$O/probe.err" || exit 11
cat "$O/probe.json"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_policy_gpu.py \
  tests/test_record_gpu.py tests/test_learner_gpu.py tests/test_fused_slot_gpu.py tests/test_drivers_gpu.py > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$O/pytest.log"; [ $rc -eq 0 ] || exit 12
timeout -k 10 600 python3 -u bench.py --legs rollout,configs --steps 5 --warmup 2 --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err"
echo "bench rc=$?"
python3 - "$O/bench.json" <<'PY'
import json, sys
s = open(sys.argv[1]).read(); d = json.loads(s[s.index('{"metric"'):])
print("policy_us", round(d["rollout"]["policy_kernel_us"], 1))
c = d["configs"]
print("c2", round(c["c2"]["d2d_iteration_s"] * 1e3, 2), round(c["c2"]["phase_ms"]["chain"], 2))
for r in c["c5"]["sweep"]:
    print("c5", r["agents"], round(r["d2d_iteration_s"] * 1e3, 2), round(r["phase_ms"]["chain"], 2))
PY
