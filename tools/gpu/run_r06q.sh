# round 6: the combinatorial actor's record policy kernels with A = 8 compile-time (D2D_POLICY_AFIX, no per-action
# range selects) and the epilogue's softmax max as one raw v_max_f32 -- probe A/B against the AFIX = 0 build
# (noafix) alternating on one box, the policy / record / update / learner / GRU tests, and the rollout + PPO legs.
# usage (GPU box): bash tools/gpu/run_r06q.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06q"; mkdir -p "$O"
run() {  # name variant
  if [ "$2" = base ]; then
    timeout -k 10 240 python3 -u tools/gpu/policy_mode_probe.py > "$O/$1.json" 2> "$O/$1.err"
  else
    D2D_LIB_VARIANT=$2 D2D_ALLOW_ABLATION=1 timeout -k 10 240 python3 -u tools/gpu/policy_mode_probe.py > "$O/$1.json" 2> "$O/$1.err"
  fi
}
for k in 1 2; do
  for v in base noafix; do run ${v}_$k $v || exit 11; cat "$O/${v}_$k.json"; done
done
timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_policy_gpu.py \
  tests/test_record_gpu.py tests/test_update_gpu.py tests/test_learner_gpu.py tests/test_gru_gpu.py tests/test_fused_slot_gpu.py \
  > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit 12
timeout -k 10 400 python3 -u bench.py --legs rollout,ppo,train --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err"
echo "bench rc=$?"
python3 - "$O/bench.json" <<'PY'
import json, sys
s = open(sys.argv[1]).read(); d = json.loads(s[s.index('{"metric"'):])
print("policy_us", round(d["rollout"]["policy_kernel_us"], 1), "upd/s", round(d["ppo"]["updates_per_s"], 1),
      "actor_ms", round(d["ppo"]["kernels"]["actor"]["ms"], 4), "train_s", d.get("train_s_per_iteration"),
      "train_phase", d.get("train", {}).get("phase_ms"))
PY
