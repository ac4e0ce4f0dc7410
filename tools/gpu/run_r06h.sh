# round 6: the policy kernel's layer-2 split residuals on v_dot2c (D2D_POLICY_SPLIT_DOT2): policy / fused-slot /
# learner tests, then A/B of the rollout slot and the configs leg (pdot0 = the and/sub split).
# usage (GPU box): bash tools/gpu/run_r06h.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06h"; mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest tests/test_policy_gpu.py tests/test_fused_slot_gpu.py tests/test_learner_gpu.py tests/test_update_gpu.py \
  -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" "$O/pytest_gpu.log" | tail -3
[ $rc -eq 0 ] || exit $rc
for k in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --legs rollout,configs --steps 5 --warmup 2 --no-cpu-baseline > "$O/new_$k.json" 2> "$O/new_$k.err" || exit 11
  D2D_LIB_VARIANT=pdot0 D2D_ALLOW_ABLATION=1 timeout -k 10 300 python3 -u bench.py --legs rollout,configs --steps 5 --warmup 2 --no-cpu-baseline > "$O/old_$k.json" 2> "$O/old_$k.err" || exit 12
done
for f in "$O"/new_*.json "$O"/old_*.json; do python3 -c "
import json; s=open('$f').read(); d=json.loads(s[s.index('{\"metric\"'):]); c=d['configs']; r=c['c5']['sweep'][-1]
print('$f'.split('/')[-1], 'policy_us', round(d['rollout']['policy_kernel_us'],1), 'c5-256', round(r['d2d_iteration_s']*1e3,1), 'chain', round(r['phase_ms']['chain'],1), 'c2', round(c['c2']['d2d_iteration_s']*1e3,1))"; done
