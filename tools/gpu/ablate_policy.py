"""Where the behaviour-policy kernel's time goes at the headline slot (64 agents x 65,536 envs,
F 30, H 64, A 8): sampling vs deterministic vs forced actions, with and without the iPPO critic.
usage (GPU box): python3 tools/gpu/ablate_policy.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "d2d-ppo_amd")]
import torch  # noqa: E402

from d2dhip.envbatch import pack_masks_torch  # noqa: E402
from d2dhip.policy import policy_mlp_step  # noqa: E402

if __name__ == "__main__":
    E, N, F, H, A = 65536, 64, 30, 64, 8
    g = torch.Generator(device="cuda").manual_seed(0)
    mk = lambda out: {"w1": torch.randn(N, H, F, device="cuda", generator=g) * 0.2,  # noqa: E731
                      "b1": torch.randn(N, H, device="cuda", generator=g) * 0.1,
                      "w2": torch.randn(N, out, H, device="cuda", generator=g) * 0.2,
                      "b2": torch.randn(N, out, device="cuda", generator=g) * 0.1}
    actor, critic = mk(A), mk(1)
    obs = torch.randint(0, 3, (E, N, F), device="cuda", generator=g).float()
    forced = pack_masks_torch(torch.randint(0, 2, (E, N, A), device="cuda", generator=g)).contiguous()
    cases = {"sample+critic": dict(critic=critic), "sample": dict(), "deterministic+critic":
             dict(critic=critic, deterministic=True), "forced": dict(forced=forced)}
    out = {}
    for name, kw in cases.items():
        for _ in range(3):
            policy_mlp_step(actor, obs, "comb", rng_step=1, **kw)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for it in range(20):
            policy_mlp_step(actor, obs, "comb", rng_step=it, **kw)
        ev[1].record()
        torch.cuda.synchronize()
        out[name] = round(ev[0].elapsed_time(ev[1]) / 20 * 1e3, 1)
    print(json.dumps({"us_per_launch": out}, indent=1))
