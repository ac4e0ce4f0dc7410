# round 5: record bit-exactness after the grid-sizing fix; the PPO update at the headline batch (65,536 envs,
# agents $1) against float64 with the relu-flip envelope
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05e"; mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests/test_record_gpu.py tests/test_update_gpu.py -m gpu -v -k "not 8192" --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" "$O/pytest.log" | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python3 -u tools/gpu/ppo_grads_full_batch.py 65536 ${1:-0:32} envelope noemu > "$O/ppo_full_65536_${1//:/-}.json" 2> "$O/ppo_full.err"
rc=$?; echo "full rc=$rc"; tail -c 600 "$O/ppo_full_65536_${1//:/-}.json"; tail -3 "$O/ppo_full.err"
exit $rc
