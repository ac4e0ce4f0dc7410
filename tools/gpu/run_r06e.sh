# round 6: single_kernel over several env groups per block (reads of the next group before the current group's
# emission): D2DEnv tests, then A/B of D2D_SINGLE_ITERS 4 (default) / 1 / 2 / 8 and the previous kernel (envprev).
# usage (GPU box): bash tools/gpu/run_r06e.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06e"; mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests/test_d2denv_gpu.py tests/test_env_gpu.py tests/test_baselines_gpu.py -m gpu -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" "$O/pytest_gpu.log" | tail -3
[ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  for v in base si1 si2 si8 envprev; do
    if [ $v = base ]; then
      timeout -k 10 200 python3 tools/gpu/single_probe.py > "$O/probe_${v}_$k.json" 2>/dev/null || exit 11
    else
      D2D_LIB_VARIANT=$v D2D_ALLOW_ABLATION=1 timeout -k 10 200 python3 tools/gpu/single_probe.py > "$O/probe_${v}_$k.json" 2>/dev/null || exit 12
    fi
    echo "$v $k $(cat $O/probe_${v}_$k.json)"
  done
done
