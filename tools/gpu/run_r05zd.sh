# round 5: central critic forward + dW1 chunked by samples (MALL reuse of the bf16 operand?) at 256 / 128 agents
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05zd"; mkdir -p "$O"
timeout -k 10 400 python3 -u tools/gpu/critic_chunk_probe.py 256 5 > "$O/chunk_256.json" 2> "$O/chunk_256.err" || exit 11
cat "$O/chunk_256.json"
