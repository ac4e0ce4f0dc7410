"""One BASELINE configs[4] D2D-PPO iteration at N agents (combinatorial, 8 channels, deadlines 7,
switch 0.8, lambda 1/14, 4,096 envs per GPU, 5 epochs), for profiling.
usage (GPU box): rocprofv3 --kernel-trace --stats -d gpurun_out/c5 -o run -- python3 tools/gpu/c5_iter.py 256"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "d2d-ppo_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

if __name__ == "__main__":
    from algorithms.d2d_ppo import D2DPPO
    from envs.combinatorial_env import CombinatorialEnv
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    p5 = dict(n_agents=N, n_channels=8, deadlines=np.full(N, 7), lbdas=np.full(N, 1 / 14), period=None,
              arrival_probs=None, offsets=None, episode_length=200, traffic_model="aperiodic",
              periodic_devices=[], channel_switch=np.ones((N, 8)) * 0.8)
    env = CombinatorialEnv(**p5, n_envs=4096, device="cuda:0", seed=22)
    torch.manual_seed(3)
    lr = D2DPPO(env, hidden_size=64, gamma=0.4, policy_lr=3e-4, value_lr=1e-3, beta_entropy=0.01,
                device=env.batch().device, useRNN=False, combinatorial=True)
    ro = lr._rollout(4096)
    upd = lr._update_state(ro)
    lr._update_epoch(ro, upd)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ro = lr._rollout(4096)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    upd = lr._update_state(ro)
    for _ in range(5):
        lr._update_epoch(ro, upd)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"N={N}: rollout {1e3 * (t1 - t0):.1f} ms; 5 epochs {1e3 * (t2 - t1):.1f} ms")
