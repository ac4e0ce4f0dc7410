# round 5: configs[4] as xp_n_agents.py writes its learner (GRU, history_len = n_agents) at the VERDICT's 4,096 envs
# (the default bench runs it at 512): rollout, first / second epoch and the 5-epoch iteration at 64 / 128 / 256 agents
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05r"; mkdir -p "$O"
timeout -k 10 1100 python3 -u bench.py --legs gru_c5 --gru-c5-envs 4096 --no-cpu-baseline --steps 5 --warmup 2 \
  > "$O/bench_gru_c5_4096.json" 2> "$O/bench_gru_c5_4096.err"
rc=$?; echo "gru_c5 rc=$rc"; tail -n 8 "$O/bench_gru_c5_4096.err"; tail -c 800 "$O/bench_gru_c5_4096.json"
exit $rc
