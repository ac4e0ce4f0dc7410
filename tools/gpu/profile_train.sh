# Kernel mix of the full-scale train leg.  usage: bash tools/gpu/profile_train.sh <tag>
R="$GRAFT_REPO_ROOT"; TAG="${1:-train}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/proftrain_$TAG" -o run --output-format csv -- \
  python3 "$R/bench.py" --legs train --steps 2 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/proftrain_$TAG.log" 2>&1
echo "rc=$?"
python3 - "$R/gpurun_out/proftrain_$TAG/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total {tot/1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} dispatches")
for r in rows[:25]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>5} {r['Percentage']:>6}%  {r['Name'][:100]}")
PY
