# round 5: the full GPU suite on the hidden-on-rows critic + occupancy-sized update grids (ABI v11)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05d"; mkdir -p "$O"
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -v --durations=30 --timeout 420 --timeout-method thread -p no:cacheprovider \
  > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" "$O/pytest_gpu.log" | tail -12
exit $rc
