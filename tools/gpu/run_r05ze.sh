# round 5 end: the 65,536-env gradient envelope re-pinned on the final kernels (two-wave critic), one agent range
# usage (GPU box): bash tools/gpu/run_r05ze.sh 0:32 | 32:64
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05ze"; mkdir -p "$O"
A="${1:-0:32}"
timeout -k 10 1000 python3 -u tools/gpu/ppo_grads_full_batch.py 65536 "$A" envelope noemu > "$O/ppo_full_65536_${A//:/-}.json" \
  2> "$O/ppo_full_${A//:/-}.err"
rc=$?; echo "full rc=$rc"; tail -c 300 "$O/ppo_full_65536_${A//:/-}.json"; tail -n 2 "$O/ppo_full_${A//:/-}.err"
exit $rc
