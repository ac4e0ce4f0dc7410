# Profile the headline kernel: trace+stats pass, then separate FETCH_SIZE and WRITE_SIZE passes.
# usage: bash tools/gpu/profile.sh <tag> [record|fp32] [commit]
R="$GRAFT_REPO_ROOT"; TAG="${1:-r01}"; MODE="${2:-record}"; COMMIT="${3:-}"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
if [ "$MODE" = record ]; then BPAS=84; else BPAS=172; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv -- \
  python3 "$R/bench.py" --legs env --env-mode "$MODE" --steps 100 --warmup 10 --no-cpu-baseline > "$R/gpurun_out/prof_$TAG.log" 2>&1 || exit 11
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch_$TAG" -o run --output-format csv -- \
  python3 "$R/bench.py" --legs env --env-mode "$MODE" --steps 20 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/pmc_fetch_$TAG.log" 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write_$TAG" -o run --output-format csv -- \
  python3 "$R/bench.py" --legs env --env-mode "$MODE" --steps 20 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/pmc_write_$TAG.log" 2>&1 || exit 13
F=$(ls "$R"/gpurun_out/pmc_fetch_$TAG/*counter_collection.csv | head -1)
W=$(ls "$R"/gpurun_out/pmc_write_$TAG/*counter_collection.csv | head -1)
python3 "$R/tools/pmc_traffic.py" "$F" "$W" "$R/gpurun_out/pmc_traffic_$TAG.json" --algorithmic-bytes $((BPAS * 64 * 65536)) --commit "$COMMIT"
