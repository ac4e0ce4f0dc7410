"""GPU parity of the GRU window-policy kernels (csrc/gru_kernels.hip) against plain torch of the same
ops: the reference's RNN module (GRU over the window from h0 = 0 -> Linear -> ReLU -> Linear ->
sigmoid / softmax / none, algorithms/ippo.py:14-51), its rollout windows (last <= L obs of the
episode, unpadded, ippo.py:302-304) and training windows (front-zero-padded to L,
preprocess_input_for_rnn ippo.py:390-403), the Bernoulli / Categorical log-probs of
PPO.select_action / evaluate (ippo.py:154-191), and the gradients of PPO.train_step's losses
(ippo.py:194-217, d2d_ppo.py:198-216) through the window (BPTT).

Both behaviour-policy kernels (exact bf16 splits, fp32 MFMA) run every policy case.
Tolerances: values 1e-5 absolute; log-probs 1e-5 absolute (or twice torch fp32's own distance to
float64, where a long window's fp32 rounding exceeds that, or two ulps of the fp32 Bernoulli
probabilities propagated through log(p) / log(1 - p)) wherever every probability is in
[1e-3, 1 - 1e-3], as the MLP kernel tests; deterministic actions exact away from ties; gradients within
2e-5 * max|g| of float64 autograd where torch fp32 itself lands in that band, else within 4x torch
fp32's distance (saturated gates / probabilities)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(params=["split", "f32"])
def policy_impl(request):
    """The behaviour-policy kernel on exact bf16 splits (default) or on fp32 MFMA
    (D2D_OPT_POLICY_F32_MFMA); the grad kernel has one implementation."""
    from d2dhip import _lib
    lib = _lib.require_gpu()
    lib.d2d_set_option(_lib.D2D_OPT_POLICY_F32_MFMA, 1 if request.param == "f32" else 0)
    yield request.param
    lib.d2d_set_option(_lib.D2D_OPT_POLICY_F32_MFMA, 0)


def make_net(N, F, H, A, seed, in_dims=None):
    from algorithms._core import RNN, StackedNets
    torch.manual_seed(seed)
    dims = in_dims or [F] * N
    st = StackedNets([RNN(d, A, H) for d in dims], dims, "rnn", "cpu")
    p = {k: v.detach().clone() for k, v in st.params.items()}
    # the reference's GRU keeps torch's default init (uniform +-1/sqrt(H)); spread it so the gates
    # leave their linear regime
    p["w_ih"] *= 2.0
    p["w_hh"] *= 2.0
    return p, dims


def make_obs(T, E, N, F, dims, seed, frac=False):
    g = torch.Generator().manual_seed(seed)
    obs = torch.zeros(T, E, N, F)
    D = max(1, F // 3)
    obs[..., :D] = torch.randint(0, 4, (T, E, N, D), generator=g).float()
    obs[..., D:] = torch.randint(-1, 2, (T, E, N, F - D), generator=g).float()
    if frac:
        obs += torch.rand(obs.shape, generator=g) * 0.3
    for k, d in enumerate(dims):
        obs[:, :, k, d:] = 0
    return obs


def gru_ref(p, obs, ep_len, L, padded, kind, dtype=torch.float64):
    """torch reference: outputs [N][T][E][A] (probs, or values [N][T][E]) of every slot's window."""
    from algorithms._core import gru_window
    T, E, N, F = obs.shape
    q = {k: v.to(dtype) for k, v in p.items()}
    outs = []
    for t in range(T):
        S = min(t % ep_len + 1, L)
        win = obs[t - S + 1: t + 1].to(dtype).permute(2, 1, 0, 3)                # [N][E][S][F]
        if padded and S < L:
            win = torch.cat([torch.zeros(N, E, L - S, F, dtype=dtype), win], 2)
        h = gru_window(win, q["w_ih"], q["w_hh"], q["b_ih"], q["b_hh"])          # [N][E][H]
        y = torch.relu(torch.baddbmm(q["b1"].unsqueeze(1), h, q["w1"].transpose(1, 2)))
        z = torch.baddbmm(q["b2"].unsqueeze(1), y, q["w2"].transpose(1, 2))        # [N][E][A]
        outs.append(torch.sigmoid(z) if kind == "sigmoid" else torch.softmax(z, -1) if kind == "softmax" else z[..., 0])
    return torch.stack(outs, 1)


CASES = [
    # kind, N, F, H, A, L, ep_len, T, E
    ("sigmoid", 3, 30, 64, 8, 6, 10, 20, 37),
    ("sigmoid", 2, 23, 16, 8, 12, 10, 20, 20),      # L > episode: every window starts at the episode start
    ("softmax", 3, 12, 32, 5, 4, 8, 16, 40),
    ("softmax", 2, 25, 64, 2, 3, 6, 12, 17),
    (None, 3, 30, 64, 1, 6, 10, 20, 37),
    (None, 2, 15, 16, 1, 5, 7, 14, 19),              # F + 1 = 16: one input tile
    ("sigmoid", 3, 46, 64, 16, 6, 10, 20, 37),      # run_ippo_combinatorial.py: 6 x 16 channels, 46 inputs
    (None, 2, 46, 64, 1, 6, 10, 20, 21),
]


@pytest.mark.parametrize("padded", [False, True])
@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}-N{c[1]}-F{c[2]}-H{c[3]}-A{c[4]}-L{c[5]}-ep{c[6]}")
def test_gru_policy_matches_torch(case, padded, policy_impl):
    from d2dhip import gru
    from d2dhip.envbatch import pack_masks_torch
    from torch.distributions import Bernoulli, Categorical
    kind, N, F, H, A, L, ep, T, E = case
    p, dims = make_net(N, F, H, A, seed=H + A)
    obs = make_obs(T, E, N, F, dims, seed=7, frac=kind == "softmax")
    ref = gru_ref(p, obs, ep, L, padded, kind)                                   # float64
    dev = "cuda"
    pd = {k: v.to(dev).contiguous() for k, v in p.items()}
    od = obs.to(dev).contiguous()
    if kind is None:
        vals = gru.policy(pd, od, None, L, ep, 0, T, padded=padded)
        got = vals.view(N, T, E).cpu().double()
        torch.testing.assert_close(got, ref, rtol=0, atol=1e-5)
        return
    g = torch.Generator().manual_seed(3)
    probs = ref                                                                  # [N][T][E][A]
    if kind == "sigmoid":
        bits = (torch.rand(N, T, E, A, generator=g) < 0.4).double()
        ref_lp = Bernoulli(probs=probs, validate_args=False).log_prob(bits).mean(-1)
        forced = pack_masks_torch(bits.permute(1, 2, 0, 3)).to(dev)              # [T][E][N]
    else:
        ids = torch.randint(0, A, (N, T, E), generator=g)
        ref_lp = Categorical(probs=probs, validate_args=False).log_prob(ids)
        forced = ids.permute(1, 2, 0).to(torch.uint8).contiguous().to(dev)
    acts, lp = gru.policy(pd, od, kind, L, ep, 0, T, padded=padded, forced=forced)
    assert torch.equal(acts, forced)
    lp = lp.view(N, T, E).cpu().double()
    well = ((probs > 1e-3) & (probs < 1 - 1e-3)).all(-1)
    assert well.float().mean() > 0.5
    # 1e-5, or twice torch fp32's own distance to float64 where a long window's fp32 rounding is larger
    with torch.no_grad():
        p32 = gru_ref(p, obs, ep, L, padded, kind, torch.float32).double()
    if kind == "sigmoid":
        lp32 = Bernoulli(probs=p32, validate_args=False).log_prob(bits).mean(-1)
    else:
        lp32 = Categorical(probs=p32, validate_args=False).log_prob(ids)
    tol = torch.clamp(2 * (lp32 - ref_lp).abs(), min=1e-5)
    if kind == "sigmoid":
        # the log-prob is taken of the fp32 probability (as torch.distributions does): two ulps of p
        # move log(1 - p) by 2 ulp(p) / (1 - p) -- up to 3e-5 in the mean at p = 0.999, where both
        # kernels sit at 1.0e-5 on one element of this case (tools/gpu/gru_diag.py)
        tol = torch.maximum(tol, (2 * 2.0 ** -23 * probs / torch.minimum(probs, 1 - probs)).mean(-1))
    err = (lp - ref_lp).abs()
    assert bool((err[well] <= tol[well]).all()), (err[well].max().item(), (err / tol)[well].max().item())
    # deterministic evaluation (ippo.py:166 / 171); one slot at a time like the rollout
    margin = (probs - 0.5).abs().min(-1).values if kind == "sigmoid" else \
        (probs.topk(2, -1).values[..., 0] - probs.topk(2, -1).values[..., 1])
    for t in (0, T // 2 + 1, T - 1):
        a_t, _ = gru.policy(pd, od, kind, L, ep, t, 1, padded=padded, deterministic=True)
        if kind == "sigmoid":
            want = pack_masks_torch((probs[:, t] > 0.5).permute(1, 0, 2))
        else:
            want = probs[:, t].argmax(-1).t().to(torch.uint8)
        clear = (margin[:, t] > 1e-5).t()                                        # [E][N]
        assert torch.equal(a_t[0].cpu()[clear], want[clear])
    # sampling: the forced evaluation of sampled actions reproduces their log-probs bit for bit
    a_s, lp_s = gru.policy(pd, od, kind, L, ep, 0, T, padded=padded, rng_step=5, seed=11)
    _, lp_f = gru.policy(pd, od, kind, L, ep, 0, T, padded=padded, forced=a_s)
    torch.testing.assert_close(lp_f, lp_s, rtol=0, atol=0)


def ref_loss_grads(p, obs, ep, L, kind, acts, logp_old, W, clip, beta, dtype):
    """autograd of the per-agent losses summed over agents (each agent's gradient is its own)."""
    from torch.distributions import Bernoulli, Categorical
    q = {k: v.to(dtype).clone().requires_grad_() for k, v in p.items()}
    out = gru_ref(q, obs, ep, L, True, kind, dtype)                            # [N][T][E](A)
    N = out.shape[0]
    if kind is None:
        loss = ((out - W.to(dtype)) ** 2).reshape(N, -1).mean(1)
        sq = ((out - W.to(dtype)) ** 2).reshape(N, -1).sum(1)
        stats = torch.stack([sq, torch.zeros_like(sq)], 1)
    else:
        if kind == "sigmoid":
            d = Bernoulli(probs=out, validate_args=False)
            logp = d.log_prob(acts.to(dtype)).mean(-1)
            ent = d.entropy().mean(-1)
        else:
            d = Categorical(probs=out, validate_args=False)
            logp = d.log_prob(acts)
            ent = d.entropy()
        ratio = torch.exp(logp - logp_old.to(dtype))
        Wd = W.to(dtype)
        s = torch.min(ratio * Wd, torch.clamp(ratio, 1 - clip, 1 + clip) * Wd)
        loss = -s.reshape(N, -1).mean(1) - beta * ent.reshape(N, -1).mean(1)
        stats = torch.stack([s.reshape(N, -1).sum(1), ent.reshape(N, -1).sum(1)], 1)
    loss.sum().backward()
    # (history_len 1: h0 = 0 is the window's only hidden input, so W_hh never enters the graph -- its gradient
    # is exactly zero)
    return ({k: v.grad if v.grad is not None else torch.zeros_like(v) for k, v in q.items()}, stats.detach(),
            out.detach())


GRAD_CASES = [
    ("sigmoid", 3, 23, 16, 8, 4, 10, 20, 20),
    ("sigmoid", 2, 30, 64, 8, 6, 8, 16, 18),
    ("softmax", 3, 12, 32, 5, 3, 6, 12, 23),
    ("softmax", 2, 15, 16, 4, 8, 6, 12, 16),         # L > episode
    (None, 3, 30, 64, 1, 5, 8, 16, 18),
    (None, 2, 12, 32, 1, 3, 6, 12, 21),
    ("sigmoid", 2, 46, 64, 16, 6, 8, 16, 18),       # run_ippo_combinatorial.py's 46 inputs: three input tiles
    (None, 2, 46, 64, 1, 6, 8, 16, 18),
    ("softmax", 2, 60, 32, 5, 4, 8, 16, 17),        # four input tiles
    ("sigmoid", 2, 30, 64, 8, 1, 8, 16, 18),        # history_len 1: no padding steps at all (cooperative path)
    (None, 2, 30, 64, 1, 1, 8, 16, 18),
]


@pytest.mark.parametrize("fmt", ["f32", "record"])
@pytest.mark.parametrize("case", GRAD_CASES, ids=lambda c: f"{c[0]}-N{c[1]}-F{c[2]}-H{c[3]}-A{c[4]}-L{c[5]}-ep{c[6]}")
def test_gru_grads_match_autograd(case, fmt):
    """fmt "record": the compact record (H = 64 with F + 1 <= 48 runs the cooperative LDS
    weight-gradient path, the other shapes the row-history kernel on the record)."""
    from d2dhip import gru
    from d2dhip.envbatch import pack_masks_torch
    kind, N, F, H, A, L, ep, T, E = case
    p, dims = make_net(N, F, H, A, seed=5 + H)
    obs = make_obs(T, E, N, F, dims, seed=9)
    g = torch.Generator().manual_seed(4)
    clip, beta = 0.1, 0.05
    with torch.no_grad():
        out64 = gru_ref(p, obs, ep, L, True, kind)
    acts = acts_dev = logp_old = None
    if kind is None:
        W = torch.randn(N, T, E, generator=g)
    else:
        if kind == "sigmoid":
            acts = (torch.rand(N, T, E, A, generator=g) < 0.4).float()
            acts_dev = pack_masks_torch(acts.permute(1, 2, 0, 3))
            lp = torch.distributions.Bernoulli(probs=out64).log_prob(acts.double()).mean(-1)
        else:
            acts = torch.randint(0, A, (N, T, E), generator=g)
            acts_dev = acts.permute(1, 2, 0).to(torch.uint8).contiguous()
            lp = torch.distributions.Categorical(probs=out64).log_prob(acts)
        logp_old = (lp + (torch.rand(N, T, E, generator=g) * 0.6 - 0.3)).float()
        W = torch.randn(N, T, E, generator=g)
    r64, s64, _ = ref_loss_grads(p, obs, ep, L, kind, acts, logp_old, W, clip, beta, torch.float64)
    r32, s32, _ = ref_loss_grads(p, obs, ep, L, kind, acts, logp_old, W, clip, beta, torch.float32)
    well = True
    dev = "cuda"
    pd = {k: v.to(dev).contiguous() for k, v in p.items()}
    # per-sample inputs in the rollout layout [T][E][N]
    W_te = W.permute(1, 2, 0).contiguous().to(dev)
    lo_te = None if logp_old is None else logp_old.permute(1, 2, 0).contiguous().to(dev)
    xin = obs.to(dev).contiguous() if fmt == "f32" else to_record(obs)
    got, stats = gru.grads(pd, xin, kind, L, ep, W_te,
                           actions=None if acts_dev is None else acts_dev.to(dev), logp_old=lo_te, clip=clip, beta=beta)
    torch.cuda.synchronize()
    for name in r64:
        gk = got[name].cpu().double()
        scale = r64[name].abs().max().item()
        err64 = (gk - r64[name]).abs().max().item()
        band = (r32[name].double() - r64[name]).abs().max().item()
        print(f"  {name}: max|g| {scale:.3e}  |kernel-f64| {err64:.2e}  |torchf32-f64| {band:.2e}")
        tol = 2e-5 * scale + 1e-7
        if band <= tol:
            assert err64 <= tol, (name, err64, tol)
        else:
            well = False
            # ill-conditioned samples (saturated gates / probabilities, where fp32 rounding of 1 - p
            # decides): within a few times torch fp32's own distance to float64
            assert err64 <= 4 * band, (name, err64, band)
    for k, d in enumerate(dims):  # padded input columns get exactly zero gradient
        assert torch.all(got["w_ih"][k, :, d:] == 0)
    # loss sums: vs float64 when well conditioned, else vs torch fp32 (log(1 - p) for p -> 1)
    st = stats.cpu().double()
    s_ref = s64 if well else s32.double()
    torch.testing.assert_close(st[:, 0], s_ref[:, 0], rtol=1e-5, atol=1e-4)
    if kind is not None:
        torch.testing.assert_close(st[:, 1], s_ref[:, 1], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("fmt", ["f32", "record"])
def test_gru_grads_bitwise_reproducible_and_large(fmt):
    """64 agents x 64-step windows (xp_load.py's history_len = n_agents) on a 4-env x 2-episode batch:
    two launches give bitwise identical gradients and loss sums (every sum is accumulated in a fixed
    order: per-wave registers, per-wave global blocks summed in wave order; no atomics), finite
    everywhere."""
    from d2dhip import gru
    from d2dhip.envbatch import pack_masks_torch
    N, F, H, A, L, ep, T, E = 64, 30, 64, 8, 64, 100, 200, 4
    p, dims = make_net(N, F, H, A, seed=1)
    obs = make_obs(T, E, N, F, dims, seed=2)
    g = torch.Generator().manual_seed(3)
    acts = pack_masks_torch((torch.rand(T, E, N, A, generator=g) < 0.3).float())
    dev = "cuda"
    pd = {k: v.to(dev).contiguous() for k, v in p.items()}
    lo = (-torch.rand(T, E, N, generator=g) * 3).to(dev)
    W = torch.randn(T, E, N, generator=g).to(dev)
    od = obs.to(dev).contiguous() if fmt == "f32" else to_record(obs)  # record: the cooperative LDS path
    g1, s1 = gru.grads(pd, od, "sigmoid", L, ep, W, actions=acts.to(dev), logp_old=lo)
    g1 = {k: v.clone() for k, v in g1.items()}
    g2, s2 = gru.grads(pd, od, "sigmoid", L, ep, W, actions=acts.to(dev), logp_old=lo)
    s1 = s1.clone()
    for k in g1:
        assert torch.isfinite(g1[k]).all()
        assert torch.equal(g1[k], g2[k]), k
    assert torch.equal(s1, s2)


# ---------------------------------------------------------------------------------------------------
# xp_load.py:78-89's configuration: hidden_size = 64, history_len = n_agents = 64 (the bench's GRU leg),
# 64 agents, 30 inputs (14 + 2 * 8), episode_length 200: T = 200 slots (a full episode) of E = 4 envs.
XP = dict(N=64, F=30, H=64, A=8, L=64, ep=200, T=200, E=4)


def window_groups(obs, ep, L, padded):
    """The windows of every slot, grouped by length: [(slots, x [N][len(slots) * E][S][F])].  Training
    windows are front-zero-padded to L (one group, ippo.py:390-403); rollout windows hold the last
    S = min(p + 1, L) obs of the episode (ippo.py:302-304), one group per S."""
    T, E, N, F = obs.shape
    pos = torch.arange(T) % ep
    S_of = torch.clamp(pos + 1, max=L)
    groups = []
    for S in ([L] if padded else sorted(set(S_of.tolist()))):
        slots = torch.arange(T) if padded else torch.nonzero(S_of == S)[:, 0]
        xs = []
        for t in slots.tolist():
            s = min(int(pos[t]) + 1, L)
            w = obs[t - s + 1: t + 1]                                                 # [s][E][N][F]
            if s < S:
                w = torch.cat([torch.zeros(S - s, E, N, F, dtype=obs.dtype, device=obs.device), w], 0)
            xs.append(w)
        x = torch.stack(xs, 0).permute(3, 0, 2, 1, 4).reshape(N, len(xs) * E, S, F)   # [N][slots*E][S][F]
        groups.append((slots, x))
    return groups


def head(q, h, kind, flip=None):
    """The RNN head; flip (bool [N][B][H]) inverts the relu mask of those (sample, unit) pairs (their
    pre-activations are within fp32 rounding of 0, so y ~ 0 either way and only the gradient's mask changes)."""
    pre = torch.baddbmm(q["b1"].unsqueeze(1), h, q["w1"].transpose(1, 2))
    y = torch.relu(pre) if flip is None else pre * ((pre > 0) ^ flip).to(pre.dtype)
    z = torch.baddbmm(q["b2"].unsqueeze(1), y, q["w2"].transpose(1, 2))
    return torch.sigmoid(z) if kind == "sigmoid" else torch.softmax(z, -1) if kind == "softmax" else z[..., 0]


def gru_ref_grouped(p, obs, ep, L, padded, kind, dtype, chunk=None):
    """gru_ref on the device, one batched GRU per window group: outputs [N][T][E](A)."""
    from algorithms._core import gru_window
    T, E, N, F = obs.shape
    q = {k: v.to(obs.device, dtype) for k, v in p.items()}
    A = q["w2"].shape[1]
    out = torch.zeros((N, T, E) + ((A,) if kind is not None else ()), dtype=dtype, device=obs.device)
    for slots, x in window_groups(obs.to(dtype), ep, L, padded):
        n = len(slots)
        o = head(q, gru_window(x, q["w_ih"], q["w_hh"], q["b_ih"], q["b_hh"]), kind)
        out[:, slots.to(obs.device)] = o.reshape((N, n, E) + o.shape[2:])
    return out


@pytest.mark.parametrize("mode", ["sampled", "deterministic", "forced_padded"])
def test_gru_policy_at_xp_load_window(mode, policy_impl):
    """gru_policy_kernel at the window the bench times (H = 64, L = 64, 64 agents, 200-slot episode)
    vs float64: the rollout's sampled mode (unpadded windows; the forced re-evaluation of the sampled
    actions reproduces their log-probs bit for bit and they match float64 to the tolerance), the
    test()-time deterministic mode (p > 0.5 decisions exact away from ties), and D2D-PPO's forced
    log-prob pass over the padded training windows."""
    xp_policy_check(mode, XP)


# xp_n_agents.py:98-112's GRU learners take history_len = n_agents: at the c5 sweep's 128 and 256 agents
# (C = 8, D = 7 -> 23 inputs) the windows are longer than the policy kernel's 63-step padding table
# (gru_kernels.hip kGruPadTab), so the padding steps run inside every window, and L = 256 > the 200-slot
# episode makes every rollout window start at the episode start.
LONG = [dict(N=128, F=23, H=64, A=8, L=128, ep=200, T=200, E=4),
        dict(N=256, F=23, H=64, A=8, L=256, ep=200, T=200, E=2)]  # (E = 2: the float64 reference takes minutes)


@pytest.mark.parametrize("c", LONG, ids=lambda c: f"N{c['N']}-L{c['L']}")
@pytest.mark.parametrize("mode", ["sampled", "deterministic", "forced_padded"])
def test_gru_policy_long_window(mode, c, policy_impl):
    """As test_gru_policy_at_xp_load_window, at history_len = n_agents = 128 / 256 (xp_n_agents); the fp32-MFMA
    A/B kernel at 128 only (the float64 reference of the 256-step windows is the suite's slowest part)."""
    if policy_impl == "f32" and c["L"] > 128:
        pytest.skip("fp32-MFMA A/B kernel: covered at L = 128")
    xp_policy_check(mode, c)


def xp_policy_check(mode, c):
    from d2dhip import gru
    from d2dhip.envbatch import pack_masks_torch
    from torch.distributions import Bernoulli
    N, F, H, A, L, ep, T, E = (c[k] for k in ("N", "F", "H", "A", "L", "ep", "T", "E"))
    p, dims = make_net(N, F, H, A, seed=21)
    dev = "cuda"
    obs = make_obs(T, E, N, F, dims, seed=22).to(dev)
    padded = mode == "forced_padded"
    with torch.no_grad():
        probs = gru_ref_grouped(p, obs, ep, L, padded, "sigmoid", torch.float64)    # [N][T][E][A]
        p32 = gru_ref_grouped(p, obs, ep, L, padded, "sigmoid", torch.float32).double()
    pd = {k: v.to(dev).contiguous() for k, v in p.items()}
    if mode == "deterministic":
        margin = (probs - 0.5).abs().min(-1).values                                  # [N][T][E]
        for t in sorted({0, 1, 63, 64, min(L, T - 1), 150, T - 1}):
            a_t, _ = gru.policy(pd, obs, "sigmoid", L, ep, t, 1, deterministic=True)
            want = pack_masks_torch((probs[:, t] > 0.5).permute(1, 0, 2))             # [E][N]
            clear = (margin[:, t] > 1e-5).t()
            assert clear.float().mean() > 0.9
            assert torch.equal(a_t[0][clear], want[clear]), t
        return
    if mode == "sampled":
        bits_te, lp = gru.policy(pd, obs, "sigmoid", L, ep, 0, T, rng_step=7, seed=13)
        _, lp_f = gru.policy(pd, obs, "sigmoid", L, ep, 0, T, forced=bits_te)
        assert torch.equal(lp_f, lp)
        from algorithms._core import unpack_actions
        bits = unpack_actions(bits_te.permute(2, 0, 1).reshape(N, -1), A).view(N, T, E, A).double()
        assert 0.05 < bits.mean().item() < 0.95
    else:
        g = torch.Generator().manual_seed(3)
        bits = (torch.rand(N, T, E, A, generator=g) < 0.4).double().to(dev)
        forced = pack_masks_torch(bits.permute(1, 2, 0, 3))                          # [T][E][N]
        acts, lp = gru.policy(pd, obs, "sigmoid", L, ep, 0, T, padded=True, forced=forced)
        assert torch.equal(acts, forced)
    lp = lp.view(N, T, E).double()
    ref_lp = Bernoulli(probs=probs, validate_args=False).log_prob(bits).mean(-1)
    lp32 = Bernoulli(probs=p32, validate_args=False).log_prob(bits).mean(-1)
    well = ((probs > 1e-3) & (probs < 1 - 1e-3)).all(-1)
    assert well.float().mean() > 0.5
    tol = torch.clamp(2 * (lp32 - ref_lp).abs(), min=1e-5)
    tol = torch.maximum(tol, (2 * 2.0 ** -23 * probs / torch.minimum(probs, 1 - probs)).mean(-1))
    err = (lp - ref_lp).abs()
    print(f"  max err {err[well].max().item():.2e}; within 1e-5: {(err[well] <= 1e-5).float().mean().item():.5f}")
    assert bool((err[well] <= tol[well]).all()), (err[well].max().item(), (err / tol)[well].max().item())


def to_record(obs):
    """The compact obs record (d2dhip/record.py) of integer-valued fp32 obs [T][E][N][F]: one byte per
    column (int8 where a column holds negatives), the bias byte 1 at column F, zeros past it."""
    from d2dhip.record import ObsRecord
    T, E, N, F = obs.shape
    R = 32 * ((F + 1 + 31) // 32)
    v = obs.round().to(torch.int32)
    assert torch.equal(v.float(), obs.float()), "record inputs must be integers"
    neg = (v < 0).reshape(-1, N, F).any(0)                                        # [N][F]
    data = torch.zeros((T, E, N, R), dtype=torch.uint8)
    data[..., :F] = (v & 0xFF).to(torch.uint8)
    data[..., F] = 1                                                                # the bias input
    sgn = torch.zeros((N, R // 32), dtype=torch.int64)
    for k in range(N):
        for c in range(F):
            if neg[k, c]:
                sgn[k, c // 32] |= 1 << (c % 32)
    sgn = torch.where(sgn >= 2 ** 31, sgn - 2 ** 32, sgn).to(torch.int32)
    return ObsRecord(data.cuda().contiguous(), F, sgn.cuda())


@pytest.fixture(params=["f32", "record", "record-history"])
def grad_input(request):
    """Rollout-buffer format of the GRU update: fp32 rows (the row-history kernel), the compact record
    (H = 64, F + 1 <= 32: the cooperative LDS weight-gradient path), or the record through the
    row-history kernel (D2D_OPT_GRU_GRAD_HISTORY)."""
    from d2dhip import _lib
    lib = _lib.require_gpu()
    lib.d2d_set_option(_lib.D2D_OPT_GRU_GRAD_HISTORY, 1 if request.param == "record-history" else 0)
    yield request.param
    lib.d2d_set_option(_lib.D2D_OPT_GRU_GRAD_HISTORY, 0)


@pytest.mark.parametrize("kind", ["sigmoid", None])
def test_gru_grads_at_xp_load_window(kind, grad_input):
    """gru_grad_kernel at the bench's window (H = 64, L = 64, 64 agents, 200-slot episode, E = 4):
    the gradients of all eight tensors vs float64 autograd over the padded training windows, with the
    fp32-band rule of test_gru_grads_match_autograd (2e-5 * max|g| where torch fp32 itself lands in
    that band, else within 4x torch fp32's distance to float64).  The reference is accumulated over
    slot chunks (every loss is a sum of per-sample terms, so chunked backward passes add up to the
    full gradient)."""
    xp_grads_check(kind, grad_input, XP["E"])


@pytest.mark.parametrize("kind", ["sigmoid", None])
def test_gru_grads_large_batch_record(kind):
    """The cooperative path keeps one accumulator per output tile across all of a wave's tiles: at 64
    envs (50 tiles x 64 steps x 4 regions of MFMA accumulation per wave) its gradients still meet the
    float64 band rule of the xp_load test."""
    xp_grads_check(kind, "record", 64)


@pytest.mark.parametrize("c", LONG, ids=lambda c: f"N{c['N']}-L{c['L']}")
@pytest.mark.parametrize("kind", ["sigmoid", None])
def test_gru_grads_long_window(kind, c, grad_input):
    """gru_grad_kernel at history_len = n_agents = 128 / 256 (xp_n_agents.py:98-112): all eight gradient
    tensors vs float64 autograd over the padded training windows, the band rule of the xp_load test.  At 256
    the product input only (the compact record, cooperative path): the float64 reference there is minutes."""
    if c["L"] > 128 and grad_input != "record" and os.environ.get("D2D_TEST_LONG_ALL") != "1":
        # (D2D_TEST_LONG_ALL=1 runs them: profiles/r05/gru_long_window_all.log)
        pytest.skip("L = 256: the record (product) path; the fp32-row and row-history kernels are covered at 128")
    xp_grads_check(kind, grad_input, c["E"], cfg=c)


LAST = []  # the last xp_grads_check's (kernel, float64, fp32) gradients


def xp_grads_check(kind, grad_input, E, check=True, cfg=None):
    """The body of test_gru_grads_at_xp_load_window at E envs; returns {tensor: (err64, band, max|g|)}
    (check=False: no assertions; tools/gpu/gru_coop_vs_history.py runs it at the bench's 256 envs)."""
    from algorithms._core import gru_window
    from d2dhip import gru
    from d2dhip.envbatch import pack_masks_torch
    from torch.distributions import Bernoulli
    c = cfg or XP
    N, F, H, A, L, ep, T = (c[k] for k in ("N", "F", "H", "A", "L", "ep", "T"))
    A = 1 if kind is None else A  # the value network: Linear(H, 1) head (the RNN critic, ippo.py:146)
    p, dims = make_net(N, F, H, A, seed=31)
    dev = "cuda"
    obs = make_obs(T, E, N, F, dims, seed=32).to(dev)
    g = torch.Generator().manual_seed(4)
    clip, beta = 0.1, 0.05
    nS = T * E
    ((_, xall),) = window_groups(obs.double(), ep, L, True)                             # [N][T*E][L][F]
    with torch.no_grad():
        out64 = gru_ref_grouped(p, obs, ep, L, True, kind, torch.float64)
    if kind is None:
        W = torch.randn(N, T, E, generator=g).to(dev)
    else:
        bits = (torch.rand(N, T, E, A, generator=g) < 0.4).double().to(dev)
        lp = Bernoulli(probs=out64, validate_args=False).log_prob(bits).mean(-1)
        logp_old = (lp + (torch.rand(N, T, E, generator=g).to(dev) * 0.6 - 0.3)).float()
        W = torch.randn(N, T, E, generator=g).to(dev)

    amb = []  # per slot chunk: the head's ambiguous relu pairs (float64 pass)

    def ref(dtype, flips=None):
        q = {k: v.to(dev, dtype).clone().requires_grad_() for k, v in p.items()}
        stats = torch.zeros(N, 2, dtype=torch.float64, device=dev)
        x = xall.to(dtype).view(N, T, E, L, F)
        for ci, t0 in enumerate(range(0, T, 25)):
            sl = slice(t0, t0 + 25)
            hL = gru_window(x[:, sl].reshape(N, -1, L, F), q["w_ih"], q["w_hh"], q["b_ih"], q["b_hh"])
            if dtype == torch.float64 and flips is None:
                # relu pairs of the head's first layer within twice the fp32 dot-product error bound of 0
                # (K = H products + bias): any fp32 evaluation may take the other mask there (the MLP
                # update's relu-flip envelope, tools/gpu/ppo_grads_full_batch.py)
                with torch.no_grad():
                    pre = torch.baddbmm(q["b1"].unsqueeze(1), hL, q["w1"].transpose(1, 2))
                    ab = torch.baddbmm(q["b1"].abs().unsqueeze(1), hL.abs(), q["w1"].abs().transpose(1, 2))
                    amb.append(pre.abs() <= 2 * (H + 2) * 2.0 ** -24 * ab)
            o = head(q, hL, kind, None if flips is None else flips[ci])
            o = o.reshape((N, 25, E) + o.shape[2:])
            if kind is None:
                sq = ((o - W[:, sl].to(dtype)) ** 2).reshape(N, -1)
                loss = sq.sum(1) / nS
                stats[:, 0] += sq.sum(1).detach().double()
            else:
                d = Bernoulli(probs=o, validate_args=False)
                ratio = torch.exp(d.log_prob(bits[:, sl].to(dtype)).mean(-1) - logp_old[:, sl].to(dtype))
                Wd = W[:, sl].to(dtype)
                sv = torch.min(ratio * Wd, torch.clamp(ratio, 1 - clip, 1 + clip) * Wd).reshape(N, -1)
                ent = d.entropy().mean(-1).reshape(N, -1)
                loss = -sv.sum(1) / nS - beta * ent.sum(1) / nS
                stats[:, 0] += sv.sum(1).detach().double()
                stats[:, 1] += ent.sum(1).detach().double()
            loss.sum().backward()
        return {k: v.grad.double() for k, v in q.items()}, stats

    r64, s64 = ref(torch.float64)
    r32, s32 = ref(torch.float32)
    n_amb = int(sum(int(m.sum()) for m in amb))
    # A kernel whose fp32 forward took the other side of an ambiguous head relu matches the float64 gradients
    # with that mask flipped.  The backward is linear in the masks given the forward, so with Delta_i = the
    # float64 gradients with agent k's i-th ambiguous head unit flipped (for every sample where it is ambiguous)
    # minus r64, the candidates of agent k are r64 + sum_{i in S} Delta_i over the subsets S of its (at most
    # four) ambiguous units; each agent is held to its nearest candidate, one subset for all eight tensors.
    units = [set() for _ in range(N)]
    for m in amb:
        for k, u in torch.nonzero(m.any(1)).tolist():
            units[k].add(u)
    units = [sorted(u) for u in units]
    n_cls = min(4, max((len(u) for u in units), default=0))
    deltas = []
    for idx in range(n_cls):
        sel = torch.zeros(N, 1, H, dtype=torch.bool, device=dev)
        for k in range(N):
            if idx < len(units[k]):
                sel[k, 0, units[k][idx]] = True
        rf = ref(torch.float64, flips=[m & sel for m in amb])[0]
        deltas.append({n: rf[n] - r64[n] for n in r64})
    subsets = [tuple(i for i in range(n_cls) if (b >> i) & 1) for b in range(1 << n_cls)]
    if n_amb:
        print(f"  {n_amb} ambiguous head relu pairs over {sum(1 for u in units if u)} agents, up to "
              f"{max(len(u) for u in units)} units per agent ({n_cls} searched)")
    pd = {k: v.to(dev).contiguous() for k, v in p.items()}
    W_te = W.permute(1, 2, 0).contiguous()
    xin = obs if grad_input == "f32" else to_record(obs.cpu())
    if kind is None:
        got, st = gru.grads(pd, xin, None, L, ep, W_te)
    else:
        got, st = gru.grads(pd, xin, "sigmoid", L, ep, W_te, actions=pack_masks_torch(bits.permute(1, 2, 0, 3)),
                            logp_old=logp_old.permute(1, 2, 0).contiguous(), clip=clip, beta=beta)
    torch.cuda.synchronize()
    well = True
    errs = {}
    LAST[:] = [got, r64, r32]  # for tools/gpu/gru_long_diag.py
    # per agent: the error of every candidate (subset S), scored over all tensors in units of their max|g|
    cand = {n: torch.stack([(got[n].double() - r64[n] - sum((deltas[i][n] for i in S), torch.zeros_like(r64[n])))
                            .abs().reshape(N, -1).amax(1) for S in subsets]) for n in r64}      # [subsets][N]
    score = torch.stack([cand[n] / r64[n].abs().max() for n in r64]).amax(0)                 # [subsets][N]
    best = score.argmin(0)                                                                      # [N]
    if n_cls:
        print(f"  agents matched with flipped head masks: {int((best > 0).sum())}")
    for name in r64:
        scale = r64[name].abs().max().item()
        err64 = cand[name].gather(0, best[None])[0].max().item()
        band = (r32[name] - r64[name]).abs().max().item()
        errs[name] = (err64, band, scale)
        print(f"  {name}: max|g| {scale:.3e}  |kernel-f64| {err64:.2e}  |torchf32-f64| {band:.2e}")
        if not check:
            continue
        tol = 2e-5 * scale + 1e-7
        if band <= tol:
            assert err64 <= tol, (name, err64, tol)
        else:
            well = False
            assert err64 <= 4 * band, (name, err64, band)
    if not check:
        return errs
    # loss sums vs float64: 1e-5 relative, or within 4x torch fp32's own distance where a long window's
    # fp32 rounding is larger (the sums over L = 256-step windows at 256 agents)
    for col in ((0,) if kind is None else (0, 1)):
        got_s, s64c, s32c = st.double()[:, col], s64[:, col], s32[:, col].double()
        tol = torch.maximum(1e-5 * s64c.abs() + 1e-4, 4 * (s32c - s64c).abs())
        assert bool(((got_s - s64c).abs() <= tol).all()), (col, ((got_s - s64c).abs() / tol).max().item())
    del well


@pytest.mark.parametrize("case", [CASES[0], CASES[1], CASES[2], CASES[4], CASES[6]],
                         ids=lambda c: f"{c[0]}-N{c[1]}-F{c[2]}-H{c[3]}-A{c[4]}-L{c[5]}-ep{c[6]}")
@pytest.mark.parametrize("deterministic", [False, True], ids=["sample", "deterministic"])
def test_gru_carried_state_equals_recompute(case, deterministic, policy_impl):
    """d2d_policy_gru_carry (ABI 14): a rollout's slots in order, each launch carrying h into the
    next while the window is a prefix extension (episode position < history_len, ippo.py:302-304), give bitwise the
    actions / log-probs / values of the per-slot recompute from h0 = 0 -- across episode boundaries, windows longer
    than the episode (L > ep_len) and past history_len, where the window slides and the launch recomputes."""
    from d2dhip import gru
    kind, N, F, H, A, L, ep, T, E = case
    p, dims = make_net(N, F, H, A, seed=H + A + 1)
    obs = make_obs(T, E, N, F, dims, seed=9, frac=kind == "softmax").to("cuda").contiguous()
    pd = {k: v.to("cuda").contiguous() for k, v in p.items()}
    hc = torch.full((gru.carry_floats(pd, E, L, ep),), float("nan"), device="cuda")
    kw = dict(seed=77, env_base=5, deterministic=deterministic)
    for t in range(T):
        pos = t % ep
        if kind is None:
            v0 = gru.policy(pd, obs, None, L, ep, t, 1)
            v1 = gru.policy(pd, obs, None, L, ep, t, 1, hcarry=hc, carry_in=1 <= pos < L)
            assert torch.equal(v0, v1), f"value, slot {t}"
        else:
            a0, l0 = gru.policy(pd, obs, kind, L, ep, t, 1, rng_step=3 + t, **kw)
            a1, l1 = gru.policy(pd, obs, kind, L, ep, t, 1, rng_step=3 + t, hcarry=hc, carry_in=1 <= pos < L, **kw)
            assert torch.equal(a0, a1), f"actions, slot {t}"
            assert torch.equal(l0, l1), f"log-probs, slot {t}"


def test_gru_carry_refuses_a_window_that_does_not_extend():
    from d2dhip import gru
    p, dims = make_net(2, 12, 16, 4, seed=1)
    pd = {k: v.to("cuda").contiguous() for k, v in p.items()}
    obs = make_obs(8, 16, 2, 12, dims, seed=1).to("cuda").contiguous()
    hc = torch.zeros((gru.carry_floats(pd, 16, 3, 8),), device="cuda")
    for slot in (0, 3, 8):  # an episode's first slot; positions >= history_len (3)
        with pytest.raises(ValueError, match="does not extend"):  # D2D_EINVAL from d2d_policy_gru_carry
            gru.policy(pd, obs, "softmax", 3, 8, slot, 1, hcarry=hc, carry_in=True)
    with pytest.raises(ValueError, match="one unpadded slot"):
        gru.policy(pd, obs, "softmax", 3, 8, 1, 2, hcarry=hc, carry_in=True)


@pytest.mark.parametrize("graph", [True, False], ids=["graph", "eager"])
def test_gru_rollout_carry_c5_256_agents(graph):
    """configs[4] as xp_n_agents.py writes its learner (D2D-PPO, GRU H = 64, history_len = N = 256 > the 200-slot
    episode: every rollout window is an episode prefix, xp_n_agents.py:98-112): the training rollout with the carried
    state (the default) equals the recompute (D2D_GRU_CARRY=0) bit for bit -- records, actions, log-probs, rewards."""
    from algorithms.d2d_ppo import D2DPPO
    from envs.combinatorial_env import CombinatorialEnv
    N, E = 256, 32
    out = []
    for carry in (False, True):
        p5 = dict(n_agents=N, n_channels=8, deadlines=np.full(N, 7), lbdas=np.full(N, 1 / 14), period=None,
                  arrival_probs=None, offsets=None, episode_length=200, traffic_model="aperiodic",
                  periodic_devices=[], channel_switch=np.ones((N, 8)) * 0.8)
        env = CombinatorialEnv(**p5, n_envs=E, device="cuda", seed=61)
        torch.manual_seed(7)
        lr = D2DPPO(env, hidden_size=64, gamma=0.4, policy_lr=3e-4, value_lr=1e-3, beta_entropy=0.01, device="cuda",
                    useRNN=True, combinatorial=True, history_len=N, early_stopping=False)
        assert lr._gru_ok()
        lr.gru_carry = carry
        lr.graph_rollout = graph
        ro = lr._rollout(E)
        torch.cuda.synchronize()
        out.append((ro.obs.data.clone(), ro.actions.clone(), ro.logp.clone(), ro.rewards.clone()))
    for x, y, name in zip(out[0], out[1], ("record", "actions", "logp", "rewards")):
        assert torch.equal(x, y), name
