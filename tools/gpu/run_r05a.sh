# round 5, first pass: the hidden-on-rows critic kernel (A/B timing and gradient difference against the
# sample-on-rows kernel), the update / record / policy / multi-rank GPU tests.
# usage (GPU box): bash tools/gpu/run_r05a.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05a"; mkdir -p "$O"
timeout -k 10 200 python3 -u tools/gpu/upd_ab.py 2048 64 > "$O/upd_ab_h64.json" 2> "$O/upd_ab.err"
rc=$?; echo "upd_ab rc=$rc"; cat "$O/upd_ab_h64.json"; [ $rc -eq 0 ] || { tail -20 "$O/upd_ab.err"; exit $rc; }
timeout -k 10 200 python3 -u tools/gpu/upd_ab.py 2048 128 > "$O/upd_ab_h128.json" 2>> "$O/upd_ab.err"
rc=$?; echo "upd_ab128 rc=$rc"; cat "$O/upd_ab_h128.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests/test_update_gpu.py tests/test_record_gpu.py tests/test_policy_gpu.py \
  tests/test_data_parallel_gpu.py -m gpu -v --durations=20 --timeout 420 --timeout-method thread -p no:cacheprovider \
  > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" "$O/pytest.log" | tail -15
exit $rc
