# round 5: the hidden-on-rows critic at 3 waves per SIMD (A/B vs the sample-on-rows kernel) + the update tests
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05b"; mkdir -p "$O"
for h in 64 128; do
  timeout -k 10 200 python3 -u tools/gpu/upd_ab.py 2048 $h > "$O/upd_ab_h$h.json" 2>> "$O/upd_ab.err"
  rc=$?; echo "upd_ab $h rc=$rc"; cat "$O/upd_ab_h$h.json"; [ $rc -eq 0 ] || { tail -20 "$O/upd_ab.err"; exit $rc; }
done
timeout -k 10 600 python3 -u -m pytest tests/test_update_gpu.py tests/test_record_gpu.py -m gpu -v --durations=10 \
  --timeout 420 --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" "$O/pytest.log" | tail -15
exit $rc
