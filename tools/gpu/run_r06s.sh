# round 6: the central critic's forward at 256 agents (S = 3,848) with more sample tiles per wave and the operand from
# registers (no LDS image: D2D_CRITIC_ST4 / KCH4 / PD -- cA 6/1/2, cB 6/2/2, cC 5/2/2, cD 5/1/3) against the product's
# LDS-image path (4 tiles, 2 chunks per iteration), alternating on one box (tools/gpu/critic_probe.py).
# usage (GPU box): bash tools/gpu/run_r06s.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06s"; mkdir -p "$O"
run() {  # name variant
  if [ "$2" = base ]; then
    timeout -k 10 300 python3 -u tools/gpu/critic_probe.py 256 10 > "$O/$1.json" 2> "$O/$1.err"
  else
    D2D_LIB_VARIANT=$2 D2D_ALLOW_ABLATION=1 timeout -k 10 300 python3 -u tools/gpu/critic_probe.py 256 10 > "$O/$1.json" 2> "$O/$1.err"
  fi
}
for k in 1 2; do
  for v in base cA cB cC cD; do run ${v}_$k $v || exit 11; echo "$v $(cat "$O/${v}_$k.json")"; done
done
