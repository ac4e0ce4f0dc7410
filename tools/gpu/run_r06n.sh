# round 6: the rollout policy kernel's actor layer 2 on fp32 MFMAs (D2D_POLICY_L2_F32 = 1 one chain, 2 two chains;
# w4: four waves per SIMD) against the split-bf16 product build, actor-only, sampled / deterministic / forced modes,
# alternating on one box; log-probs saved for an offline comparison.
# usage (GPU box): bash tools/gpu/run_r06n.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06n"; mkdir -p "$O"
run() {  # name variant
  if [ "$2" = base ]; then
    timeout -k 10 240 python3 -u tools/gpu/policy_mode_probe.py --save "$O/$1.pt" > "$O/$1.json" 2> "$O/$1.err"
  else
    D2D_LIB_VARIANT=$2 D2D_ALLOW_ABLATION=1 timeout -k 10 240 python3 -u tools/gpu/policy_mode_probe.py --save "$O/$1.pt" \
      > "$O/$1.json" 2> "$O/$1.err"
  fi
}
for k in 1 2; do
  for v in base l2f1 l2f2 l2f1w4 l2f2w4; do run ${v}_$k $v || exit 11; cat "$O/${v}_$k.json"; done
done
