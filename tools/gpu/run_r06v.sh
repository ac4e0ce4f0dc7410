# round 6, final kernels: kernel-trace stats of one c5 256-agent D2D-PPO iteration (tools/gpu/c5_iter.py) -- the forced
# log-prob pass, chain, actor / critic kernels at configs[4]'s widest state.
# usage (GPU box): bash tools/gpu/run_r06v.sh
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/r06v"; mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/c5_256" -o run --output-format csv -- python3 "$R/tools/gpu/c5_iter.py" 256 \
  > "$O/c5_256.log" 2>&1
rc=$?; echo "rc=$rc"; tail -2 "$O/c5_256.log"
cp "$(ls "$O"/c5_256/*kernel_stats.csv | head -1)" "$O/c5_256_kernel_stats.csv" 2>/dev/null
rm -rf "$O/c5_256"
exit $rc
