# kernel-level profile of the rollout and PPO legs
R="$GRAFT_REPO_ROOT"; TAG="${1:-legs}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv -- \
  python3 "$R/bench.py" --legs env,rollout,ppo --steps 5 --warmup 2 --rollout-steps 20 --ppo-epochs 3 --no-cpu-baseline > "$R/gpurun_out/prof_$TAG.log" 2>&1
echo "rc=$?"
head -25 "$R/gpurun_out/prof_$TAG/run_kernel_stats.csv" | cut -c1-200
