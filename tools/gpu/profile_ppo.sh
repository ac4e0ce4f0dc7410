# Kernel mix of the PPO-update leg.  usage: bash tools/gpu/profile_ppo.sh <tag>
R="$GRAFT_REPO_ROOT"; TAG="${1:-ppo}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/profppo_$TAG" -o run --output-format csv -- \
  python3 "$R/bench.py" --legs ppo --steps 3 --warmup 1 --ppo-epochs 3 --no-cpu-baseline > "$R/gpurun_out/profppo_$TAG.log" 2>&1
echo "rc=$?"
python3 - "$R/gpurun_out/profppo_$TAG/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total {tot/1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} dispatches")
for r in rows[:25]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>5} {r['Percentage']:>6}%  {r['Name'][:100]}")
PY
