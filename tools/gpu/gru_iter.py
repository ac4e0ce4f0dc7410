"""One xp_load-configuration D2D-PPO iteration with GRU policies (bench.py's GRU leg (3): 64 agents x 8
channels, H = 64, history_len = 64, 256 envs, 5 epochs), for profiling.
usage (GPU box): rocprofv3 --kernel-trace --stats -d gpurun_out/gru_iter -o run -- python3 tools/gpu/gru_iter.py [E] [history]
("history": the row-history update kernel, D2D_OPT_GRU_GRAD_HISTORY, for A/B timing)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "d2d-ppo_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

if __name__ == "__main__":
    import bench
    from algorithms.d2d_ppo import D2DPPO
    from envs.combinatorial_env import CombinatorialEnv
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    if "history" in sys.argv[2:]:
        from d2dhip import _lib
        _lib.require_gpu().d2d_set_option(_lib.D2D_OPT_GRU_GRAD_HISTORY, 1)
    params = bench.config3_params(200)
    env = CombinatorialEnv(**params, n_envs=E, device="cuda:0", seed=52)
    torch.manual_seed(6)
    np.random.seed(6)
    lr = D2DPPO(env, hidden_size=64, gamma=0.6, policy_lr=3e-4, value_lr=1e-3, device=env.batch().device,
                useRNN=True, combinatorial=True, history_len=64, early_stopping=False)
    for it in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ro = lr._rollout(E)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        upd = lr._update_state(ro)
        for _ in range(5):
            lr._update_epoch(ro, upd)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"GRU D2D-PPO E={E}: rollout {1e3 * (t1 - t0):.1f} ms; 5 epochs {1e3 * (t2 - t1):.1f} ms")
