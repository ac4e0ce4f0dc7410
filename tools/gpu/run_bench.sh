# Full GPU pass: gpu tests, bench (all legs), profiles.  usage: bash tools/gpu/run_bench.sh <tag>
R="$GRAFT_REPO_ROOT"; TAG="${1:-r01}"
cd "$R" || exit 9
mkdir -p gpurun_out
timeout -k 10 1000 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -2
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1
brc=$?; echo "bench rc=$brc"; tail -c 3000 gpurun_out/bench_$TAG.log
[ $brc -eq 0 ] || exit $brc
bash tools/gpu/profile.sh "$TAG"; echo "profile rc=$?"
