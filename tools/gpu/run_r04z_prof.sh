# round-4 end, part 1 (profiles, stamped with the code commit): rocprofv3 kernel-trace stats of the env leg
# (the headline kernel's duration), FETCH_SIZE / WRITE_SIZE passes -> HBM traffic per launch, and the SQ
# counter passes -> MFMA busy / VALU per MFMA of the update, policy and GRU kernels.
# usage (GPU box): bash tools/gpu/run_r04z_prof.sh <commit>
R="$GRAFT_REPO_ROOT"; COMMIT="$1"; cd "$R" || exit 9
O="$R/gpurun_out/r04z"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/env_stats" -o run --output-format csv -- \
  python3 "$R/bench.py" --legs env --env-mode record --steps 200 --warmup 20 --no-cpu-baseline > "$O/env_under_rocprof.json" 2>&1
rc=$?; echo "env stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run --output-format csv -- \
  python3 "$R/bench.py" --legs env --env-mode record --steps 20 --warmup 5 --no-cpu-baseline > "$O/pmc_fetch.log" 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o run --output-format csv -- \
  python3 "$R/bench.py" --legs env --env-mode record --steps 20 --warmup 5 --no-cpu-baseline > "$O/pmc_write.log" 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
F=$(ls "$O"/pmc_fetch/*counter_collection.csv | head -1)
W=$(ls "$O"/pmc_write/*counter_collection.csv | head -1)
python3 "$R/tools/pmc_traffic.py" "$F" "$W" "$O/pmc_traffic_record.json" --algorithmic-bytes $((84 * 64 * 65536)) \
  --commit "$COMMIT" --kernel comb_kernel --envs 65536 --agents 64
rc=$?; echo "traffic rc=$rc"; [ $rc -eq 0 ] || exit $rc
cp "$F" "$O/pmc_fetch_counter_collection.csv"; cp "$W" "$O/pmc_write_counter_collection.csv"
cp "$(ls "$O"/env_stats/*kernel_stats.csv | head -1)" "$O/env_record_kernel_stats.csv"
bash "$R/tools/gpu/pmc_mfma.sh" r04z "$COMMIT"
rc=$?; echo "pmc_mfma rc=$rc"; [ $rc -eq 0 ] || exit $rc
cp "$R/gpurun_out/pmcm_r04z/pmc_mfma.json" "$O/pmc_mfma.json"
cp "$(ls "$R"/gpurun_out/pmcm_r04z/stats/*kernel_stats.csv | head -1)" "$O/pmc_legs_kernel_stats.csv"
rm -rf "$R/gpurun_out/pmcm_r04z" "$O/env_stats" "$O/pmc_fetch" "$O/pmc_write"
exit 0
