# round 4: GRU policy at small batches on 4-wave workgroups -- GRU policy / learner tests and the xp_load iteration
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04u"; mkdir -p "$O"
timeout -k 10 200 python3 tools/gpu/gru_iter.py 256 > "$O/gru_iter.log" 2>&1
echo "gru_iter rc=$? $(grep 'GRU D2D' "$O/gru_iter.log" | tail -2 | tr '\n' ' ')"
timeout -k 10 500 python3 -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gru_gpu.py \
  tests/test_learner_gpu.py tests/test_drivers_gpu.py -k "policy or rnn or gru or driver or xp" > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 "$O/pytest.log")"; grep FAILED "$O/pytest.log" | head
exit $rc
