"""One BASELINE configs[1] D2D-PPO iteration (chsel 16 agents x 4 channels, 4,096 envs, 5 epochs),
timed after a warm-up: wall clock vs summed GPU kernel time shows how launch-bound it is.
usage (GPU box): rocprofv3 --kernel-trace --stats -d gpurun_out/c2 -o run -- python3 tools/gpu/c2_iter.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "d2d-ppo_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


class A:
    episode_length = 200


if __name__ == "__main__":
    from envs.channel_selection_env import ChannelSelectionEnv
    N = 16
    p2 = dict(n_agents=N, n_channels=4, deadlines=np.full(N, 7), lbdas=np.full(N, 1 / 3.5), period=np.full(N, 2),
              arrival_probs=np.full(N, 0.5), offsets=np.zeros(N), episode_length=200,
              traffic_model="aperiodic", periodic_devices=[], channel_switch=np.full(5, 0.8))
    env = ChannelSelectionEnv(**p2, n_envs=4096, device="cuda:0", seed=21)
    it_s, fused = bench._d2d_iteration(env, 5, combinatorial=False)
    from algorithms.d2d_ppo import D2DPPO
    torch.manual_seed(3)
    lr = D2DPPO(env, hidden_size=64, gamma=0.4, policy_lr=3e-4, value_lr=1e-3, beta_entropy=0.01,
                device=env.batch().device, useRNN=False, combinatorial=False)
    for _ in range(2):
        lr._rollout(4096)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ro = lr._rollout(4096)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    upd = lr._update_state(ro)
    lr._update_epoch(ro, upd)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"iteration {it_s * 1e3:.2f} ms (fused={fused}); rollout {1e3 * (t1 - t0):.2f} ms; one epoch {1e3 * (t2 - t1):.2f} ms")
