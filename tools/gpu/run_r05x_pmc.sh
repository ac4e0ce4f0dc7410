# round 5: per-leg PMC profiles of the MFMA kernels (tools/gpu/pmc_legs.sh; rollout, ppo, gru_slot, gru legs alone)
# usage (GPU box): bash tools/gpu/run_r05x_pmc.sh <commit>
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05x"; mkdir -p "$O"
bash tools/gpu/pmc_legs.sh r05 "$1" > "$O/pmc_legs.log" 2>&1
rc=$?; echo "pmc rc=$rc"; tail -n 5 "$O/pmc_legs.log"; ls "$R/gpurun_out/pmcl_r05"
exit $rc
