"""D2D-PPO central critic at small state widths: one training iteration (rollout + 5
epochs) of BASELINE configs[1] (chsel 16 agents x 4 channels, S = 117) and of configs[4] at 8 / 16 agents
(S = 128 / 248), 4,096 envs, with the critic on torch fp32 (CRITIC_SPLIT_MIN_DIM = 256, the round-3
default for these widths) and on the bf16 split GEMMs (threshold 0), phase split from bench.PhaseTimer.
usage (GPU box): python3 tools/gpu/critic_small.py [min_dim ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "d2d-ppo_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def envs():
    from envs.channel_selection_env import ChannelSelectionEnv
    from envs.combinatorial_env import CombinatorialEnv
    N = 16
    p2 = dict(n_agents=N, n_channels=4, deadlines=np.full(N, 7), lbdas=np.full(N, 1 / 3.5), period=np.full(N, 2),
              arrival_probs=np.full(N, 0.5), offsets=np.zeros(N), episode_length=200,
              traffic_model="aperiodic", periodic_devices=[], channel_switch=np.full(5, 0.8))
    yield "c2", (lambda: ChannelSelectionEnv(**p2, n_envs=4096, device="cuda:0", seed=21)), False
    for N in (8, 16, 32):
        p5 = dict(n_agents=N, n_channels=8, deadlines=np.full(N, 7), lbdas=np.full(N, 1 / 14), period=None,
                  arrival_probs=None, offsets=None, episode_length=200, traffic_model="aperiodic",
                  periodic_devices=[], channel_switch=np.ones((N, 8)) * 0.8)
        yield f"c5_{N}", (lambda p5=p5: CombinatorialEnv(**p5, n_envs=4096, device="cuda:0", seed=22)), True


if __name__ == "__main__":
    from algorithms.d2d_ppo import D2DPPO
    dims = [int(a) for a in sys.argv[1:]] or [256, 0]
    out = {}
    for name, make, comb in envs():
        for md in dims:
            D2DPPO.CRITIC_SPLIT_MIN_DIM = md
            env = make()
            it_s, fused, phases = bench._d2d_iteration(env, 5, combinatorial=comb)
            rec = {"iteration_ms": it_s * 1e3, "phase_ms": {k: round(v, 3) for k, v in phases.items()}}
            out[f"{name}/min_dim={md}"] = rec
            print(name, md, json.dumps(rec), flush=True)
            del env
            torch.cuda.empty_cache()
    print(json.dumps(out))
