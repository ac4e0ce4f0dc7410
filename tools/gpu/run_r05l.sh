# round 5: 65,536-env gradient envelope agents 32-63; the c5 GRU bench leg alone
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05l"; mkdir -p "$O"
timeout -k 10 600 python3 -u tools/gpu/ppo_grads_full_batch.py 65536 32:64 envelope noemu > "$O/ppo_full_65536_32-64.json" 2> "$O/ppo_full.err"
rc=$?; echo "full rc=$rc"; tail -c 300 "$O/ppo_full_65536_32-64.json"; tail -n 2 "$O/ppo_full.err"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 450 python3 -u bench.py --legs gru_c5 --no-cpu-baseline --steps 5 --warmup 2 > "$O/bench_gru_c5.json" 2> "$O/bench_gru_c5.err"
rc=$?; echo "bench rc=$rc"; tail -c 1500 "$O/bench_gru_c5.json"; tail -n 5 "$O/bench_gru_c5.err"
exit $rc
