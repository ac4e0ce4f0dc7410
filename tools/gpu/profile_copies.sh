# Attribute __amd_rocclr_copyBuffer dispatches (blit kernels of hipMemcpy*) in the PPO leg:
# kernel trace + HIP API trace + memory-copy trace (no PMC counters in this pass).
# usage: bash tools/gpu/profile_copies.sh <tag>
R="$GRAFT_REPO_ROOT"; TAG="${1:-copies}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --stats -d "$R/gpurun_out/profcp_$TAG" \
  -o run --output-format csv -- python3 "$R/bench.py" --legs ppo --steps 3 --warmup 1 --ppo-epochs 3 \
  --no-cpu-baseline > "$R/gpurun_out/profcp_$TAG.log" 2>&1
rc=$?; echo "rc=$rc"
python3 - "$R/gpurun_out/profcp_$TAG" <<'PY'
import csv, glob, os, sys
d = sys.argv[1]
for pat in ("*kernel_stats.csv", "*hip_api_stats.csv", "*memory_copy_stats.csv"):
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        rows = list(csv.DictReader(open(f)))
        print("==", os.path.basename(f))
        for r in rows[:14]:
            print(f"  x{r.get('Calls', '?'):>6} {float(r.get('TotalDurationNs', 0)) / 1e6:9.3f} ms  {r.get('Name', '')[:90]}")
PY
exit $rc
