# D2DEnv single_kernel (envs/env.py) at 64 agents x 65,536 envs, one obs format per pass set (the d2denv leg's
# --d2denv-env-only --env-mode fp32 / record: every single_kernel dispatch is that format's launch): kernel-trace stats,
# then separate FETCH_SIZE and WRITE_SIZE passes (MI355X_MICROARCH.md HBM recipe), summarised by tools/pmc_traffic.py
# against the leg's algorithmic bytes per launch (bench.py d2denv_leg: fp32 rows 567.5 MB -> pmc_traffic_single.json,
# the compact record 282.3 MB -> pmc_traffic_single_record.json).
# usage (GPU box): bash tools/gpu/profile_single.sh <tag> <commit>
R="$GRAFT_REPO_ROOT"; TAG="${1:-single}"; COMMIT="${2:-}"
cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/prof_$TAG"; mkdir -p "$O"
for mode in fp32 record; do
  if [ "$mode" = fp32 ]; then ALG=567541760; OUT=pmc_traffic_single.json; else ALG=282329088; OUT=pmc_traffic_single_record.json; fi
  BARGS=(--legs d2denv --d2denv-env-only --steps 5 --warmup 2 --no-cpu-baseline --env-mode $mode)
  D="$O/$mode"; mkdir -p "$D"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$D/stats" -o run --output-format csv -- \
    python3 "$R/bench.py" "${BARGS[@]}" > "$D/stats.log" 2>&1 || exit 11
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex single_kernel -d "$D/fetch" -o run --output-format csv -- \
    python3 "$R/bench.py" "${BARGS[@]}" > "$D/fetch.log" 2>&1 || exit 12
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex single_kernel -d "$D/write" -o run --output-format csv -- \
    python3 "$R/bench.py" "${BARGS[@]}" > "$D/write.log" 2>&1 || exit 13
  F=$(ls "$D"/fetch/*counter_collection.csv | head -1)
  W=$(ls "$D"/write/*counter_collection.csv | head -1)
  python3 "$R/tools/pmc_traffic.py" "$F" "$W" "$O/$OUT" --kernel single_kernel --envs 65536 --agents 64 \
    --algorithmic-bytes $ALG --commit "$COMMIT" || exit 14
  cp "$(ls "$D"/stats/*kernel_stats.csv | head -1)" "$O/single_${mode}_kernel_stats.csv"
done
