# round 6: the rollout policy kernel with the paired epilogue's Philox block drawn before the tile MFMAs
# (D2D_POLICY_RNG_EARLY, rngE) and with every actor-only record instantiation built for four waves per SIMD (w4), against
# the product build, alternating on one box (tools/gpu/policy_mode_probe.py).
# usage (GPU box): bash tools/gpu/run_r06w.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06w"; mkdir -p "$O"
run() {  # name variant
  if [ "$2" = base ]; then
    timeout -k 10 240 python3 -u tools/gpu/policy_mode_probe.py > "$O/$1.json" 2> "$O/$1.err"
  else
    D2D_LIB_VARIANT=$2 D2D_ALLOW_ABLATION=1 timeout -k 10 240 python3 -u tools/gpu/policy_mode_probe.py > "$O/$1.json" 2> "$O/$1.err"
  fi
}
for k in 1 2; do
  for v in base rngE w4; do run ${v}_$k $v || exit 11; cat "$O/${v}_$k.json"; done
done
