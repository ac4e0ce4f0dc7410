# round 6: LLVM's max-ILP machine scheduler (-mllvm -amdgpu-sched-strategy=max-ilp) on the GRU (gilp), policy (pilp) and
# update (uilp) kernels, A/B against the product build, alternating on one box.
# usage (GPU box): bash tools/gpu/run_r06l.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06l"; mkdir -p "$O"
run() {  # name variant legs
  if [ "$2" = base ]; then
    timeout -k 10 400 python3 -u bench.py --legs "$3" --steps 5 --warmup 2 --no-cpu-baseline > "$O/$1.json" 2> "$O/$1.err"
  else
    D2D_LIB_VARIANT=$2 D2D_ALLOW_ABLATION=1 timeout -k 10 400 python3 -u bench.py --legs "$3" --steps 5 --warmup 2 --no-cpu-baseline > "$O/$1.json" 2> "$O/$1.err"
  fi
}
for k in 1 2; do
  run gru_base_$k base gru || exit 11
  run gru_gilp_$k gilp gru || exit 12
  run mlp_base_$k base rollout,ppo || exit 13
  run mlp_pilp_$k pilp rollout,ppo || exit 14
  run mlp_uilp_$k uilp rollout,ppo || exit 15
done
for f in "$O"/*.json; do python3 -c "
import json; s=open('$f').read(); d=json.loads(s[s.index('{\"metric\"'):]); n='$f'.split('/')[-1]
if 'gru' in d: g=d['gru']; print(n, 'slot', round(g['policy_slot']['ms'],2), 'update', round(g['update']['ms'],2), 'iter', round(g['d2d_iteration_s'],4))
else: print(n, 'policy_us', round(d['rollout']['policy_kernel_us'],1), 'actor', round(d['ppo']['kernels']['actor']['ms'],4), 'critic', round(d['ppo']['kernels']['critic']['ms'],4), 'upd/s', round(d['ppo']['updates_per_s'],1))"; done
