# GPU test pass: pytest -m gpu (single process), log under gpurun_out/
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 1000 python -m pytest tests -m gpu -q -p no:cacheprovider -k "${1:-}" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
exit $rc
