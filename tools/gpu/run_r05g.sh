# round 5: actor dZ split once + packed dH mask: A/B timing, record / update tests; then the envelope agents 32-63
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05g"; mkdir -p "$O"
timeout -k 10 200 python3 -u tools/gpu/upd_ab.py 2048 64 > "$O/upd_ab_h64.json" 2>> "$O/upd_ab.err"
rc=$?; echo "upd_ab rc=$rc"; cat "$O/upd_ab_h64.json"; [ $rc -eq 0 ] || { tail -20 "$O/upd_ab.err"; exit $rc; }
timeout -k 10 300 python3 -u -m pytest tests/test_record_gpu.py tests/test_update_gpu.py -m gpu -v -k "not 8192" --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" "$O/pytest.log" | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u tools/gpu/ppo_grads_full_batch.py 65536 32:64 envelope noemu > "$O/ppo_full_65536_32-64.json" 2> "$O/ppo_full.err"
rc=$?; echo "full rc=$rc"; tail -2 "$O/ppo_full.err"
exit $rc
