# round 4: policy kernel with the fused critic vs actor + value launches, with and without one-round sizing
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04m"; mkdir -p "$O"
for sz in 1 2 3 1 2 3; do
  D2D_POLICY_SIZING=$sz timeout -k 10 200 python3 tools/gpu/policy_split_probe.py > "$O/probe_sz$sz.json" 2> "$O/probe_sz$sz.err"
  rc=$?; [ $rc -eq 0 ] || { echo "probe rc=$rc"; tail -5 "$O/probe_sz$sz.err"; exit $rc; }
  echo "sizing=$sz $(cat "$O/probe_sz$sz.json")"
done
