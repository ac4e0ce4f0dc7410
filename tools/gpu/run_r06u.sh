# round 6: the PPO update grids with at least R resident rounds of workgroups (D2D_UPD_MIN_ROUNDS = 1 (product), 3, 4, 6)
# at the PPO leg's 2,048-env batch and at the train leg's headline batch, alternating on one box.
# usage (GPU box): bash tools/gpu/run_r06u.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06u"; mkdir -p "$O"
for k in 1 2; do
  for r in 1 3 4 6; do
    D2D_UPD_MIN_ROUNDS=$r timeout -k 10 300 python3 -u bench.py --legs ppo --steps 10 --warmup 3 --no-cpu-baseline \
      > "$O/ppo_r${r}_$k.json" 2> "$O/ppo_r${r}_$k.err" || exit 11
    python3 - "$O/ppo_r${r}_$k.json" $r <<'PY'
import json, sys
s = open(sys.argv[1]).read(); d = json.loads(s[s.index('{"metric"'):])
p = d["ppo"]
print("rounds", sys.argv[2], "upd/s", round(p["updates_per_s"], 1), "actor", round(p["kernels"]["actor"]["ms"], 4),
      "critic", round(p["kernels"]["critic"]["ms"], 4))
PY
  done
done
