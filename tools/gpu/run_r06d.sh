# round 6: single_kernel with the gather codes prefetched (A/B against the previous env kernel, envprev variant),
# the dW1 kernel with narrow-state tiles (tests + configs leg).
# usage (GPU box): bash tools/gpu/run_r06d.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06d"; mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests/test_critic_dw1_gpu.py tests/test_d2denv_gpu.py tests/test_learner_gpu.py -k "dw1 or central_critic or d2d or single or D2DEnv or d2denv" -m gpu -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" "$O/pytest_gpu.log" | tail -3
[ $rc -eq 0 ] || exit $rc
for k in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --legs d2denv --d2denv-env-only --steps 5 --warmup 2 --no-cpu-baseline --env-mode record > "$O/single_new_$k.json" 2>&1 || exit 11
  D2D_LIB_VARIANT=envprev D2D_ALLOW_ABLATION=1 timeout -k 10 300 python3 -u bench.py --legs d2denv --d2denv-env-only --steps 5 --warmup 2 --no-cpu-baseline --env-mode record > "$O/single_prev_$k.json" 2>&1 || exit 12
done
for f in "$O"/single_*.json; do python3 -c "
import json,sys; s=open('$f').read(); d=json.loads(s[s.index('{\"metric\"'):]); print('$f'.split('/')[-1], round(d['d2denv']['kernel_avg_us'],1), round(d['d2denv']['hbm_frac'],3))"; done
timeout -k 10 400 python3 -u bench.py --legs configs --steps 5 --warmup 2 --no-cpu-baseline > "$O/bench_configs.json" 2> "$O/bench_configs.err"
rc=$?; echo "bench rc=$rc"
exit $rc
