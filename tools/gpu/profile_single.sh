# D2DEnv single_kernel (envs/env.py) at 64 agents x 65,536 envs: kernel-trace stats, then separate FETCH_SIZE and
# WRITE_SIZE passes (MI355X_MICROARCH.md HBM recipe), summarised by tools/pmc_traffic.py against the d2denv leg's
# algorithmic bytes per launch (bench.py d2denv_leg: 567.5 MB).
# usage (GPU box): bash tools/gpu/profile_single.sh <tag> <commit>
R="$GRAFT_REPO_ROOT"; TAG="${1:-single}"; COMMIT="${2:-}"
cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/prof_$TAG"; mkdir -p "$O"
BARGS=(--legs d2denv --d2denv-env-only --steps 5 --warmup 2 --no-cpu-baseline --env-mode record)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/stats" -o run --output-format csv -- \
  python3 "$R/bench.py" "${BARGS[@]}" > "$O/stats.log" 2>&1 || exit 11
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex single_kernel -d "$O/fetch" -o run --output-format csv -- \
  python3 "$R/bench.py" "${BARGS[@]}" > "$O/fetch.log" 2>&1 || exit 12
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex single_kernel -d "$O/write" -o run --output-format csv -- \
  python3 "$R/bench.py" "${BARGS[@]}" > "$O/write.log" 2>&1 || exit 13
F=$(ls "$O"/fetch/*counter_collection.csv | head -1)
W=$(ls "$O"/write/*counter_collection.csv | head -1)
python3 "$R/tools/pmc_traffic.py" "$F" "$W" "$O/pmc_traffic_single.json" --kernel single_kernel --envs 65536 --agents 64 \
  --algorithmic-bytes 567541760 --commit "$COMMIT" || exit 14
