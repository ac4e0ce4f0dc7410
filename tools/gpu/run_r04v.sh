# round 4: D2D central critic GEMM orientation probe (256 agents)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04v"; mkdir -p "$O"
timeout -k 10 200 python3 tools/gpu/critic_gemm_probe.py > "$O/critic_gemm.json" 2> "$O/critic_gemm.err"
rc=$?; echo "rc=$rc"; cat "$O/critic_gemm.json"; [ $rc -eq 0 ] || tail -3 "$O/critic_gemm.err"
exit $rc
