import sys, os
sys.path[:0] = ["/root/repo", "/root/repo/d2d-ppo_amd", "/root/repo/tests"]
import torch
from torch.distributions import Bernoulli
from test_gru_gpu import make_net, make_obs, gru_ref
from d2dhip import gru, _lib
from d2dhip.envbatch import pack_masks_torch
kind, N, F, H, A, L, ep, T, E = ("sigmoid", 2, 23, 16, 8, 12, 10, 20, 20)
p, dims = make_net(N, F, H, A, seed=H + A)
obs = make_obs(T, E, N, F, dims, seed=7)
ref = gru_ref(p, obs, ep, L, False, kind)
p32 = gru_ref(p, obs, ep, L, False, kind, torch.float32).double()
g = torch.Generator().manual_seed(3)
bits = (torch.rand(N, T, E, A, generator=g) < 0.4).double()
ref_lp = Bernoulli(probs=ref, validate_args=False).log_prob(bits).mean(-1)
lp32 = Bernoulli(probs=p32, validate_args=False).log_prob(bits).mean(-1)
forced = pack_masks_torch(bits.permute(1, 2, 0, 3)).to("cuda")
pd = {k: v.cuda().contiguous() for k, v in p.items()}
lib = _lib.require_gpu()
res = {}
for impl in (0, 1):
    lib.d2d_set_option(_lib.D2D_OPT_POLICY_F32_MFMA, impl)
    _, lp = gru.policy(pd, obs.cuda().contiguous(), kind, L, ep, 0, T, padded=False, forced=forced)
    res[impl] = lp.view(N, T, E).cpu().double()
well = ((ref > 1e-3) & (ref < 1 - 1e-3)).all(-1)
tol = torch.clamp(2 * (lp32 - ref_lp).abs(), min=1e-5)
for impl in (0, 1):
    err = (res[impl] - ref_lp).abs()
    r = (err / tol)[well]
    print("impl", impl, "max err", err[well].max().item(), "top err/tol", r.topk(5).values.tolist())
d = (res[0] - res[1]).abs()
print("split vs f32 max", d.max().item(), "mean", d.mean().item())
i = ((res[0] - ref_lp).abs() * well).argmax()
idx = torch.unravel_index(i, well.shape)
print("worst", [int(x) for x in idx], "probs", ref[idx].tolist(), "lp ref", ref_lp[idx].item(), "split", res[0][idx].item(), "f32", res[1][idx].item(), "torch32", lp32[idx].item())
