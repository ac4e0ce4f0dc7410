# round 6: the D2DEnv single_kernel's FETCH / WRITE traffic per obs format (fp32 rows and the compact record, each its
# own pass set: tools/gpu/profile_single.sh) -- the earlier pass mixed the two formats' launches in one median.
# usage (GPU box): bash tools/gpu/run_r06t.sh <commit>
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
bash tools/gpu/profile_single.sh r06t "$1" > "$R/gpurun_out/profile_single_r06t.log" 2>&1
rc=$?; echo "profile rc=$rc"; tail -3 "$R/gpurun_out/profile_single_r06t.log"
cat "$R/gpurun_out/prof_r06t/pmc_traffic_single.json"; echo; cat "$R/gpurun_out/prof_r06t/pmc_traffic_single_record.json"
rm -rf "$R/gpurun_out/prof_r06t/fp32" "$R/gpurun_out/prof_r06t/record"
exit $rc
