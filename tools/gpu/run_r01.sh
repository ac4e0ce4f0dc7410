cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 400 python bench.py --steps 200 --warmup 20 > gpurun_out/bench.log 2>&1
  brc=$?
  echo "bench rc=$brc"; tail -3 gpurun_out/bench.log
  if [ $brc -eq 0 ]; then
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r01" -o run --output-format csv -- python3 "$R/bench.py" --steps 100 --warmup 10 --no-cpu-baseline > "$R/gpurun_out/prof_r01.log" 2>&1
    echo "rocprof rc=$?"
  fi
fi
