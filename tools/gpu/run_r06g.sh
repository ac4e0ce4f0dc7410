# round 6: D2D-PPO epochs on two streams (forced pass beside the critic forward, critic backward beside the actor
# gradients): equality test + A/B of the configs leg (D2D_OVERLAP=1 / 0); D2DEnv record with pre-decoded codes.
# usage (GPU box): bash tools/gpu/run_r06g.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06g"; mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest tests/test_update_gpu.py tests/test_d2denv_gpu.py tests/test_learner_gpu.py -k "side_stream or record or d2d or D2D" \
  -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" "$O/pytest_gpu.log" | tail -3
[ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 400 python3 -u bench.py --legs configs,d2denv --steps 5 --warmup 2 --no-cpu-baseline > "$O/bench_ov1_$k.json" 2> "$O/bench_ov1_$k.err" || exit 11
  D2D_OVERLAP=0 timeout -k 10 400 python3 -u bench.py --legs configs --steps 5 --warmup 2 --no-cpu-baseline > "$O/bench_ov0_$k.json" 2> "$O/bench_ov0_$k.err" || exit 12
done
for f in "$O"/bench_ov*.json; do python3 -c "
import json; s=open('$f').read(); d=json.loads(s[s.index('{\"metric\"'):]); c=d['configs']
print('$f'.split('/')[-1], 'c2', round(c['c2']['d2d_iteration_s']*1e3,1), 'c5', [(r['agents'], round(r['d2d_iteration_s']*1e3,1)) for r in c['c5']['sweep']], 'd2denv rec', round(d['d2denv']['record']['kernel_avg_us'],1) if 'd2denv' in d else '')"; done
