# round 6: the fp32-row env traffic profile stamped with the code commit, and the c5 GRU leg's epoch phase split.
# usage (GPU box): bash tools/gpu/run_r06k.sh <commit>
R="$GRAFT_REPO_ROOT"; COMMIT="$1"; cd "$R" || exit 9
O="$R/gpurun_out/r06k"; mkdir -p "$O"
bash tools/gpu/profile.sh r06k fp32 "$COMMIT" > "$O/profile_fp32.log" 2>&1
rc=$?; echo "fp32 traffic rc=$rc"; tail -2 "$O/profile_fp32.log"; [ $rc -eq 0 ] || exit $rc
cp "$R/gpurun_out/pmc_traffic_r06k.json" "$O/pmc_traffic_fp32.json"
cp "$(ls "$R"/gpurun_out/prof_r06k/*kernel_stats.csv | head -1)" "$O/env_fp32_kernel_stats.csv"
rm -rf "$R/gpurun_out/prof_r06k" "$R/gpurun_out/pmc_fetch_r06k" "$R/gpurun_out/pmc_write_r06k"
cd "$R"
timeout -k 10 600 python3 -u bench.py --legs gru_c5 --steps 5 --warmup 2 --no-cpu-baseline > "$O/bench_gru_c5.json" 2> "$O/bench_gru_c5.err"
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; s=open('$O/bench_gru_c5.json').read(); d=json.loads(s[s.index('{\"metric\"'):])
for r in d['gru_c5']['sweep']: print(r['agents'], round(r['epoch_s'],3), {k: round(v,1) for k,v in r['epoch_phase_ms'].items()})"
exit $rc
