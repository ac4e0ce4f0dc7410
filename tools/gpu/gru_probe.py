"""Run the GRU kernels once at the bench's GRU shapes (for rocprofv3 --kernel-trace / --pmc passes).
usage: python tools/gpu/gru_probe.py [grad|policy|both]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "d2d-ppo_amd")]
import torch  # noqa: E402

from d2dhip import gru  # noqa: E402
from d2dhip.envbatch import pack_masks_torch  # noqa: E402


def net(N, F, H, A, dev):
    g = torch.Generator().manual_seed(0)
    r = lambda *s: (torch.rand(*s, generator=g) * 0.4 - 0.2).to(dev)  # noqa: E731
    return {"w_ih": r(N, 3 * H, F), "w_hh": r(N, 3 * H, H), "b_ih": r(N, 3 * H), "b_hh": r(N, 3 * H),
            "w1": r(N, H, H), "b1": r(N, H), "w2": r(N, A, H), "b2": r(N, A)}


def main(which):
    dev = "cuda"
    N, F, H, A, L = 64, 30, 64, 8, 64
    if which in ("grad", "both"):
        T, E = 200, 256
        p = net(N, F, H, A, dev)
        obs = torch.randint(0, 3, (T, E, N, F), device=dev).float()
        acts = pack_masks_torch((torch.rand(T, E, N, A, device=dev) < 0.3).float())
        lo = -torch.rand(T, E, N, device=dev) * 3
        W = torch.randn(T, E, N, device=dev)
        for _ in range(2):
            gru.grads(p, obs, "sigmoid", L, T, W, actions=acts, logp_old=lo)
        torch.cuda.synchronize()
    if which in ("policy", "both"):
        T, E = L, 65536
        p = net(N, F, H, A, dev)
        obs = torch.randint(0, 3, (T, E, N, F), device=dev).float()
        for _ in range(2):
            gru.policy(p, obs, "sigmoid", L, 200, L - 1, 1, rng_step=3, seed=1)
        torch.cuda.synchronize()
    print("probe done", which)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "both")
