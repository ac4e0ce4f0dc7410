# round 6: the forced-mode policy pass (D2D-PPO's epoch-start log-probs): 32-bit forced-word offsets and no action
# store (actions = NULL) in the product build, against a timing-only variant without the forced-word DMA (fab),
# alternating on one box.
# usage (GPU box): bash tools/gpu/run_r06o.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06o"; mkdir -p "$O"
run() {  # name variant
  if [ "$2" = base ]; then
    timeout -k 10 240 python3 -u tools/gpu/policy_mode_probe.py > "$O/$1.json" 2> "$O/$1.err"
  else
    D2D_LIB_VARIANT=$2 D2D_ALLOW_ABLATION=1 timeout -k 10 240 python3 -u tools/gpu/policy_mode_probe.py > "$O/$1.json" 2> "$O/$1.err"
  fi
}
for k in 1 2; do
  for v in base fab; do run ${v}_$k $v || exit 11; cat "$O/${v}_$k.json"; done
done
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_policy_gpu.py tests/test_record_gpu.py \
  > "$O/pytest.log" 2>&1; echo "pytest rc=$?"; tail -3 "$O/pytest.log"
