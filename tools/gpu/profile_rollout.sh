R="$GRAFT_REPO_ROOT"; TAG="${1:-rollout}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv -- \
  python3 "$R/bench.py" --legs env,rollout --steps 5 --warmup 2 --rollout-steps 20 --no-cpu-baseline > "$R/gpurun_out/prof_$TAG.log" 2>&1
echo "rc=$?"
python3 - "$R/gpurun_out/prof_$TAG/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print(f"{float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4} {r['Percentage']:>6}%  {r['Name'][:90]}")
PY
grep -E "policy_mlp|comb_kernel" "$R/gpurun_out/prof_$TAG/run_kernel_trace.csv" | head -2 | cut -d, -f12-22
