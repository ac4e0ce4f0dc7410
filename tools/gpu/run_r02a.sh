# round-2 pass A: multi-env learner parity + test() parity + c5 sizes, data-parallel rehearsal,
# default bench (new CPU legs, per-phase train timing), copyBuffer attribution
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29541 tools/gpu/rehearse_dp.py > gpurun_out/rehearse_dp.log 2>&1
rc=$?; echo "rehearse_dp rc=$rc"; grep rehearse_dp gpurun_out/rehearse_dp.log | cut -c1-600
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu/profile_copies.sh r02a
