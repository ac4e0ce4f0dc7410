"""Phase split of the D2DEnv step kernel (single_kernel, csrc/env_kernels.hip) at the bench's d2denv workload (64 agents,
ring neighbourhoods, 65,536 envs): the step with the fp32 obs rows (the product), without any obs output (the env
step + state stores alone), and the obs emission's share by difference.  HIP-event time per launch, median of reps.
usage (GPU box): python tools/gpu/single_probe.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "d2d-ppo_amd")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from envs.env import D2DEnv
    N, E = 64, 65536
    nb = [[(k - 1) % N, k, (k + 1) % N] for k in range(N)]
    env = D2DEnv(n_agents=N, deadlines=np.full(N, 7), lbdas=np.full(N, 1 / 14), episode_length=200,
                 channel_switch=0.2, neighbourhoods=nb, n_envs=E, device="cuda:0", seed=31)
    b = env.batch()
    act = b.action_buffer()
    b.reset(want_obs=True)
    out = {}
    for name, want in (("obs", True), ("no_obs", False), ("obs2", True), ("no_obs2", False)):
        ts = []
        for _ in range(60):
            if b.timestep >= 200:
                b.reset(want_obs=True)
            b.sample_actions(0.05, out=act)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            b.step(act, want_obs=want)
            e1.record()
            ts.append((e0, e1))
        torch.cuda.synchronize()
        out[name] = float(np.median([a.elapsed_time(c) for a, c in ts[10:]]) * 1e3)
    print(json.dumps({"single_probe_us": out}))


if __name__ == "__main__":
    main()
