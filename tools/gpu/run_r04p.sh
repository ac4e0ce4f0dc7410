# round 4: kernel-level profile of one c5 D2D-PPO iteration at 256 agents (critic forward / chain phases)
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/r04p"; mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/c5_256" -o run --output-format csv -- python3 "$R/tools/gpu/c5_iter.py" 256 > "$O/c5_256.log" 2>&1
rc=$?; echo rc=$rc; tail -2 "$O/c5_256.log"
S=$(ls "$O"/c5_256/*kernel_stats.csv | head -1); cp "$S" "$O/c5_256_kernel_stats.csv"
python3 - "$O/c5_256_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:25]:
    print(r['Name'][:100], r['Calls'], round(float(r['TotalDurationNs']) / 1e6, 2), 'ms', round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
rm -rf "$O/c5_256"
exit $rc
