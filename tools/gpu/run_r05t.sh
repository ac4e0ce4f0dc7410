# round 5: critic_t at 2 waves per SIMD (no spills) vs 3 (18 VGPRs spilled), real-rollout A/B, alternating
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05t"; mkdir -p "$O"
for k in 1 2; do
  timeout -k 10 300 python3 -u tools/gpu/upd_ab.py 2048 64 10 real > "$O/ab_w3_$k.json" 2> "$O/ab_w3_$k.err" || exit 11
  D2D_LIB_VARIANT=critt2 D2D_ALLOW_ABLATION=1 timeout -k 10 300 python3 -u tools/gpu/upd_ab.py 2048 64 10 real \
    > "$O/ab_w2_$k.json" 2> "$O/ab_w2_$k.err" || exit 12
  python3 -c "
import json
for n in ('w3', 'w2'):
    d = json.loads(open('$O/ab_' + n + '_$k.json').read())
    print(n, $k, 'critic_t', round(d['critic_t_ms'], 4), 'actor', round(d['actor_ms'], 4))"
done
