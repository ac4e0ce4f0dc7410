# 2-rank rehearsal of bench.py's N>1 path on a 1-GPU box (gloo, both ranks on cuda:0).
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
mkdir -p gpurun_out
D2D_BENCH_BACKEND=gloo D2D_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 5 \
  --envs 16384 --rollout-steps 10 --ppo-envs 512 --ppo-epochs 2 --no-cpu-baseline > gpurun_out/rehearse2.log 2>&1
rc=$?; echo "rc=$rc"; grep '^{"metric"' gpurun_out/rehearse2.log | cut -c1-1500; tail -5 gpurun_out/rehearse2.log | cut -c1-300
exit $rc
