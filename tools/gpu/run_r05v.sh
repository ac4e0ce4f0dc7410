# round 5: rollout policy kernel (actor-only record instantiation) at 4 waves per SIMD (128 VGPRs) vs 3, alternating
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05v"; mkdir -p "$O"
for k in 1 2; do
  timeout -k 10 300 python3 -u bench.py --legs rollout --steps 20 --warmup 5 --no-cpu-baseline \
    > "$O/w3_$k.json" 2> "$O/w3_$k.err" || exit 11
  D2D_LIB_VARIANT=pol4 D2D_ALLOW_ABLATION=1 timeout -k 10 300 python3 -u bench.py --legs rollout --steps 20 --warmup 5 \
    --no-cpu-baseline > "$O/w4_$k.json" 2> "$O/w4_$k.err" || exit 12
  python3 -c "
import json
for n in ('w3', 'w4'):
    d = json.loads(open('$O/' + n + '_$k.json').read().strip().splitlines()[-1])['rollout']
    print(n, $k, 'policy_us', round(d['policy_kernel_us'], 2), 'env_us', round(d['env_kernel_us'], 2))"
done
