# round 5: c5 as xp_n_agents writes it (GRU, history_len = N) at the VERDICT's 4,096 envs, on the padding-region BPTT
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05zc"; mkdir -p "$O"
timeout -k 10 1080 python3 -u bench.py --legs gru_c5 --gru-c5-envs 4096 --no-cpu-baseline > "$O/bench_gru_c5_4096.json" \
  2> >(tee "$O/bench_gru_c5_4096.log" >&2)
rc=$?; echo "rc=$rc"; tail -c 700 "$O/bench_gru_c5_4096.json"; exit $rc
