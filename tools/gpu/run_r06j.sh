# round 6: fused Adam for the stacked learners (D2D_FUSED_ADAM): learner / update / driver / data-parallel tests,
# then A/B of the PPO leg and the train leg.
# usage (GPU box): bash tools/gpu/run_r06j.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06j"; mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest tests/test_learner_gpu.py tests/test_update_gpu.py tests/test_drivers_gpu.py tests/test_gru_gpu.py \
  tests/test_data_parallel_gpu.py -k "not large_rollout" -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" "$O/pytest_gpu.log" | tail -3
[ $rc -eq 0 ] || exit $rc
for k in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --legs ppo,train --steps 5 --warmup 2 --no-cpu-baseline > "$O/fused_$k.json" 2> "$O/fused_$k.err" || exit 11
  D2D_FUSED_ADAM=0 timeout -k 10 300 python3 -u bench.py --legs ppo,train --steps 5 --warmup 2 --no-cpu-baseline > "$O/foreach_$k.json" 2> "$O/foreach_$k.err" || exit 12
done
for f in "$O"/fused_*.json "$O"/foreach_*.json; do python3 -c "
import json; s=open('$f').read(); d=json.loads(s[s.index('{\"metric\"'):]); p=d['ppo']
print('$f'.split('/')[-1], 'ppo ms', round(p['ms_per_update'],3), {k: round(v,3) for k,v in p['phase_ms_per_update'].items()}, 'train s', round(d['train_s_per_iteration'],4))"; done
