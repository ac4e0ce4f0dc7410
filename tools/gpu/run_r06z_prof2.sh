# round-6 end, profiles stamped with the code commit: rocprofv3 kernel-trace stats of the env leg (the headline
# kernel's duration), FETCH_SIZE / WRITE_SIZE passes -> HBM traffic per launch, then the per-leg SQ counter passes
# of the MFMA kernels (tools/gpu/pmc_legs.sh: rollout, ppo, gru_slot, gru legs alone).
# usage (GPU box): bash tools/gpu/run_r06z_prof2.sh <commit>
R="$GRAFT_REPO_ROOT"; COMMIT="$1"; cd "$R" || exit 9
O="$R/gpurun_out/r06z_prof2"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/env_stats" -o run --output-format csv -- \
  python3 "$R/bench.py" --legs env --env-mode record --steps 200 --warmup 20 --no-cpu-baseline > "$O/env_under_rocprof.json" 2>&1
rc=$?; echo "env stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run --output-format csv -- \
  python3 "$R/bench.py" --legs env --env-mode record --steps 20 --warmup 5 --no-cpu-baseline > "$O/pmc_fetch.log" 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o run --output-format csv -- \
  python3 "$R/bench.py" --legs env --env-mode record --steps 20 --warmup 5 --no-cpu-baseline > "$O/pmc_write.log" 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
F=$(ls "$O"/pmc_fetch/*counter_collection.csv | head -1)
W=$(ls "$O"/pmc_write/*counter_collection.csv | head -1)
python3 "$R/tools/pmc_traffic.py" "$F" "$W" "$O/pmc_traffic_record.json" --algorithmic-bytes $((84 * 64 * 65536)) \
  --commit "$COMMIT" --kernel comb_kernel --envs 65536 --agents 64
rc=$?; echo "traffic rc=$rc"; [ $rc -eq 0 ] || exit $rc
cp "$F" "$O/pmc_fetch_counter_collection.csv"; cp "$W" "$O/pmc_write_counter_collection.csv"
cp "$(ls "$O"/env_stats/*kernel_stats.csv | head -1)" "$O/env_record_kernel_stats.csv"
rm -rf "$O/env_stats" "$O/pmc_fetch" "$O/pmc_write"
bash "$R/tools/gpu/pmc_legs.sh" r06 "$COMMIT" > "$O/pmc_legs.log" 2>&1
rc=$?; echo "pmc legs rc=$rc"; tail -n 3 "$O/pmc_legs.log"; [ $rc -eq 0 ] || exit $rc
for leg in rollout ppo gru_slot gru; do
  cp "$R/gpurun_out/pmcl_r06/pmc_mfma_$leg.json" "$O/pmc_mfma_$leg.json"
  cp "$(ls "$R/gpurun_out/pmcl_r06/$leg/stats/"*kernel_stats.csv | head -1)" "$O/${leg}_kernel_stats.csv"
done
bash "$R/tools/gpu/profile_single.sh" r06z2 "$COMMIT" > "$O/profile_single.log" 2>&1
rc=$?; echo "single traffic rc=$rc"; [ $rc -eq 0 ] || exit $rc
cp "$R"/gpurun_out/prof_r06z2/pmc_traffic_single*.json "$R"/gpurun_out/prof_r06z2/single_*_kernel_stats.csv "$O/"
rm -rf "$R/gpurun_out/prof_r06z2/fp32" "$R/gpurun_out/prof_r06z2/record"
rm -rf "$R/gpurun_out/pmcl_r06" "$R/gpurun_out/prof_r06z2"
exit 0
