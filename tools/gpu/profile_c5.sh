R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/c5_256" -o run --output-format csv -- python3 "$R/tools/gpu/c5_iter.py" 256 > "$R/gpurun_out/c5_256.log" 2>&1
echo rc=$?; tail -2 "$R/gpurun_out/c5_256.log"
