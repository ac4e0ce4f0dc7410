# round 6: one forced-word DMA per tile pair (D2D_POLICY_FORCED_PAIR, product) against one per tile (fpair0),
# alternating on one box; the policy / record / update / learner tests; the configs leg (c2, c5 chain phases).
# usage (GPU box): bash tools/gpu/run_r06r.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06r"; mkdir -p "$O"
run() {  # name variant
  if [ "$2" = base ]; then
    timeout -k 10 240 python3 -u tools/gpu/policy_mode_probe.py > "$O/$1.json" 2> "$O/$1.err"
  else
    D2D_LIB_VARIANT=$2 D2D_ALLOW_ABLATION=1 timeout -k 10 240 python3 -u tools/gpu/policy_mode_probe.py > "$O/$1.json" 2> "$O/$1.err"
  fi
}
for k in 1 2; do
  for v in base fpair0; do run ${v}_$k $v || exit 11; cat "$O/${v}_$k.json"; done
done
timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_policy_gpu.py \
  tests/test_record_gpu.py tests/test_update_gpu.py tests/test_learner_gpu.py \
  > "$O/pytest.log" 2>&1
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
