"""GPU parity of the fused PPO-update kernels (csrc/update_kernels.hip) against plain torch
autograd of the same losses (the reference's PPO.train_step: evaluate + clipped surrogate +
entropy bonus, algorithms/ippo.py:178-217, d2d_ppo.py:198-216; critic MSE ippo.py:210-216),
run on the CPU in float64 (the exact-math baseline) and float32 (the reference precision).

Tolerance: every gradient tensor within 2e-5 * max|g| (+1e-7) of the float64 result, which
is the band the torch fp32 gradients themselves land in (asserted alongside), whenever every
probability is in [1e-4, 1 - 1e-4]; otherwise (samples at torch's eps clamp or with p -> 1,
where fp32 rounding decides) within 4x torch fp32's own distance to float64.  Loss sums
within 1e-5 relative.  Inputs: reference initialisation (orthogonal, gain 2), env-like
integer observations (the bf16-exact path) or fractional ones (the six-term split path),
ratios spread over and beyond the clip range, ragged env counts (E not a multiple of 32),
heterogeneous observation widths (zero-padded columns must get exactly zero gradient)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def make_nets(N, F, H, A, in_dims, seed, critic):
    from algorithms._core import Policy, StackedNets, Value
    torch.manual_seed(seed)
    dims = in_dims or [F] * N
    if critic:
        st = StackedNets([Value(d, H) for d in dims], dims, "mlp", "cpu")
    else:
        st = StackedNets([Policy(d, A, H) for d in dims], dims, "mlp", "cpu", act="softmax")
    return {k: v.detach().clone() for k, v in st.params.items()}, dims


def make_obs(T, E, N, F, dims, seed, frac):
    g = torch.Generator().manual_seed(seed)
    obs = torch.zeros(T, E, N, F)
    D = max(1, F // 3)
    obs[..., :D] = torch.randint(0, 4, (T, E, N, D), generator=g).float()
    obs[..., D:] = torch.randint(-1, 2, (T, E, N, F - D), generator=g).float()
    if frac:
        obs += torch.rand(obs.shape, generator=g) * 0.4
    for k, d in enumerate(dims):
        obs[:, :, k, d:] = 0
    return obs


def forward_probs(net, x):
    """x [N][B][F] -> softmax probs [N][B][A] (Policy.forward, ippo.py:69-75)."""
    h = torch.relu(torch.baddbmm(net["b1"].unsqueeze(1), x, net["w1"].transpose(1, 2)))
    return torch.softmax(torch.baddbmm(net["b2"].unsqueeze(1), h, net["w2"].transpose(1, 2)), -1)


def ref_actor(net, obs, acts_f, logp_old, W, kind, clip, beta, dtype):
    from torch.distributions import Bernoulli, Categorical
    p = {k: v.to(dtype).clone().requires_grad_() for k, v in net.items()}
    T, E, N, F = obs.shape
    x = obs.to(dtype).permute(2, 0, 1, 3).reshape(N, T * E, F)
    probs = forward_probs(p, x)
    if kind == "comb":
        d = Bernoulli(probs=probs, validate_args=False)
        logp = d.log_prob(acts_f.to(dtype)).mean(-1)
        ent = d.entropy().mean(-1)
    else:
        d = Categorical(probs=probs, validate_args=False)
        logp = d.log_prob(acts_f)
        ent = d.entropy()
    ratio = torch.exp(logp - logp_old.to(dtype))
    Wd = W.to(dtype)
    s = torch.min(ratio * Wd, torch.clamp(ratio, 1 - clip, 1 + clip) * Wd)
    loss = -s.mean(1) - beta * ent.mean(1)
    loss.sum().backward()
    return {k: v.grad for k, v in p.items()}, s.sum(1), ent.sum(1), logp.detach()


def ref_critic(net, obs, R, dtype):
    p = {k: v.to(dtype).clone().requires_grad_() for k, v in net.items()}
    T, E, N, F = obs.shape
    x = obs.to(dtype).permute(2, 0, 1, 3).reshape(N, T * E, F)
    h = torch.relu(torch.baddbmm(p["b1"].unsqueeze(1), x, p["w1"].transpose(1, 2)))
    v = torch.baddbmm(p["b2"].unsqueeze(1), h, p["w2"].transpose(1, 2))[..., 0]
    loss = ((v - R.to(dtype)) ** 2).mean(1)
    loss.sum().backward()
    return {k: v.grad for k, v in p.items()}, ((v - R.to(dtype)) ** 2).sum(1)


def conditioned(probs, lo=1e-4):
    """Every probability of every sample away from torch's eps clamp and from 1: there the
    float64 gradient is the exact-math baseline.  Near the clamp (p ~ 1.2e-7, where the
    gradient jumps between ~1 and 0) or near p -> 1 (1 - p loses its digits in fp32) both
    fp32 implementations follow their own rounding, so only the fp32 comparison is made."""
    return bool(probs.min() > lo and probs.max() < 1 - lo)


def assert_grads(got, ref64, ref32, dims, F, well_conditioned=True):
    for name in ref64:
        g = got[name].cpu().double()
        r = ref64[name]
        scale = r.abs().max().item()
        err64 = (g - r).abs().max().item()
        err32 = (g - ref32[name].double()).abs().max().item()
        band = (ref32[name].double() - r).abs().max().item()   # torch fp32's own error
        print(f"  {name}: max|g| {scale:.3e}  |kernel-f64| {err64:.2e}  |kernel-f32| {err32:.2e}  "
              f"|torchf32-f64| {band:.2e}")
        if well_conditioned:
            tol = 2e-5 * scale + 1e-7
            assert band <= tol, (name, "fp32 torch outside the band", band, tol)
            assert err64 <= tol, (name, err64, tol)
        else:
            # ill-conditioned samples: the kernel stays within a few times torch fp32's own error
            tol = max(4 * band, 2e-5 * scale) + 1e-7
            assert err64 <= tol, (name, err64, tol)
    if dims is not None:  # padded input columns: exactly zero
        for k, d in enumerate(dims):
            assert torch.all(got["w1"][k, :, d:] == 0)


CASES = [
    # kind, N, T, E, F, H, A, in_dims, frac
    ("comb", 4, 3, 100, 30, 64, 8, None, False),
    ("comb", 7, 2, 64, 30, 64, 8, [23, 30, 23, 30, 23, 30, 30], False),
    ("comb", 3, 2, 45, 46, 32, 16, None, True),
    ("comb", 2, 4, 33, 10, 20, 3, None, False),
    ("chsel", 3, 3, 70, 12, 64, 5, None, True),
    ("chsel", 5, 2, 96, 24, 64, 16, [24, 20, 24, 21, 24], False),
    ("chsel", 2, 1, 17, 40, 48, 9, None, True),
    # configs[4] (xp_n_agents sweep) shapes bench.py times: 128 / 256 agents, C = 8, D = 7 -> F = 23
    ("comb", 128, 2, 72, 23, 64, 8, None, False),
    ("comb", 256, 2, 40, 23, 64, 8, None, False),
    # the learners' default hidden_size 128 (ippo.py:225) and the modules' default 100: 8 hidden tiles
    ("comb", 4, 3, 100, 30, 128, 8, None, False),
    ("chsel", 3, 2, 70, 12, 128, 5, None, True),
    ("comb", 3, 2, 45, 23, 100, 8, [23, 20, 23], False),
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}-N{c[1]}-T{c[2]}-E{c[3]}-F{c[4]}-H{c[5]}-A{c[6]}"
                                              f"{'-het' if c[7] else ''}{'-frac' if c[8] else ''}" for c in CASES])
def test_actor_grad_matches_autograd(case):
    from d2dhip.envbatch import pack_masks_torch
    from d2dhip.update import actor_grads
    kind, N, T, E, F, H, A, dims, frac = case
    net, dims_ = make_nets(N, F, H, A, dims, seed=3, critic=False)
    obs = make_obs(T, E, N, F, dims_, seed=5, frac=frac)
    g = torch.Generator().manual_seed(9)
    B = T * E
    if kind == "comb":
        acts_f = (torch.rand(N, B, A, generator=g) < 0.4).float()
        masks = pack_masks_torch(acts_f.view(N, T, E, A).permute(1, 2, 0, 3).contiguous())  # [T][E][N]
        acts_dev = masks
    else:
        acts_f = torch.randint(0, A, (N, B), generator=g)
        acts_dev = acts_f.view(N, T, E).permute(1, 2, 0).to(torch.uint8).contiguous()
    with torch.no_grad():
        x = obs.permute(2, 0, 1, 3).reshape(N, B, F).double()
        probs = forward_probs({k: v.double() for k, v in net.items()}, x)
        if kind == "comb":
            lp = torch.distributions.Bernoulli(probs=probs).log_prob(acts_f.double()).mean(-1)
        else:
            lp = torch.distributions.Categorical(probs=probs).log_prob(acts_f)
    # ratios spread over [0.7, 1.35]: inside and on both sides of the clip range
    logp_old = (lp + (torch.rand(N, B, generator=g) * 0.6 - 0.3)).float()
    W = torch.randn(N, B, generator=g)
    clip, beta = 0.1, 0.05
    r64, s64, e64, _ = ref_actor(net, obs, acts_f, logp_old, W, kind, clip, beta, torch.float64)
    r32, s32, e32, _ = ref_actor(net, obs, acts_f, logp_old, W, kind, clip, beta, torch.float32)
    dev = "cuda"
    netd = {k: v.to(dev).contiguous() for k, v in net.items()}
    # logp_old in the rollout layout [T][E][N]; W in the learners' env-major [N][E*T] layout
    lo_te = logp_old.view(N, T, E).permute(1, 2, 0).contiguous().to(dev)
    W_env_major = W.view(N, T, E).permute(0, 2, 1).reshape(N, E * T).contiguous().to(dev)
    grads, stats = actor_grads(netd, obs.to(dev).contiguous(), acts_dev.to(dev), lo_te, W_env_major, kind,
                               clip=clip, beta=beta)
    torch.cuda.synchronize()
    well = conditioned(probs)
    assert_grads(grads, r64, r32, dims, F, well)
    st = stats.cpu().double()
    # loss sums: vs float64 when well conditioned, else vs torch fp32 (log(1 - p) for p -> 1)
    s_ref, e_ref = (s64, e64) if well else (s32.double(), e32.double())
    assert torch.allclose(st[:, 0], s_ref, rtol=1e-5, atol=1e-4), (st[:, 0], s_ref)
    assert torch.allclose(st[:, 1], e_ref, rtol=1e-5, atol=1e-4), (st[:, 1], e_ref)


@pytest.mark.parametrize("case", [c for c in CASES if c[0] == "comb"],
                         ids=lambda c: f"N{c[1]}-T{c[2]}-E{c[3]}-F{c[4]}-H{c[5]}{'-frac' if c[8] else ''}")
def test_critic_grad_matches_autograd(case):
    from d2dhip.update import critic_grads
    _, N, T, E, F, H, _, dims, frac = case
    net, dims_ = make_nets(N, F, H, 1, dims, seed=4, critic=True)
    obs = make_obs(T, E, N, F, dims_, seed=6, frac=frac)
    g = torch.Generator().manual_seed(2)
    R = torch.randn(N, T * E, generator=g)
    r64, l64 = ref_critic(net, obs, R, torch.float64)
    r32, _ = ref_critic(net, obs, R, torch.float32)
    dev = "cuda"
    netd = {k: v.to(dev).contiguous() for k, v in net.items()}
    R_te = R.view(N, T, E).permute(1, 2, 0).contiguous().to(dev)   # [T][E][N] (GAE output layout)
    grads, stats = critic_grads(netd, obs.to(dev).contiguous(), R_te)
    torch.cuda.synchronize()
    assert_grads(grads, r64, r32, dims, F)
    assert torch.allclose(stats.cpu().double()[:, 0], l64, rtol=1e-5, atol=1e-4)


def test_update_deterministic_and_large():
    """64 x 8 at 256 envs x 20 slots: bitwise-identical on repeat; fp32-band vs float64 autograd."""
    from d2dhip.envbatch import pack_masks_torch
    from d2dhip.update import actor_grads
    N, T, E, F, H, A = 64, 20, 256, 30, 64, 8
    net, dims = make_nets(N, F, H, A, None, seed=1, critic=False)
    obs = make_obs(T, E, N, F, dims, seed=2, frac=False)
    g = torch.Generator().manual_seed(3)
    B = T * E
    acts_f = (torch.rand(N, B, A, generator=g) < 0.3).float()
    masks = pack_masks_torch(acts_f.view(N, T, E, A).permute(1, 2, 0, 3).contiguous())
    logp_old = -torch.rand(N, B, generator=g) * 3
    W = torch.randn(N, B, generator=g)
    r64, _, _, _ = ref_actor(net, obs, acts_f, logp_old, W, "comb", 0.1, 0.01, torch.float64)
    r32, _, _, _ = ref_actor(net, obs, acts_f, logp_old, W, "comb", 0.1, 0.01, torch.float32)
    with torch.no_grad():
        probs = forward_probs({k: v.double() for k, v in net.items()}, obs.permute(2, 0, 1, 3).reshape(N, B, F).double())
    dev = "cuda"
    netd = {k: v.to(dev).contiguous() for k, v in net.items()}
    # [N][T*E] time-major -> strided [T][E][N] views (no copy: the kernel takes element strides)
    lo_v = logp_old.to(dev).view(N, T, E).permute(1, 2, 0)
    W_v = W.to(dev).view(N, T, E).permute(1, 2, 0)
    args = (netd, obs.to(dev).contiguous(), masks.to(dev), lo_v, W_v, "comb")
    g1, s1 = actor_grads(*args)
    g1 = {k: v.clone() for k, v in g1.items()}
    s1 = s1.clone()
    g2, s2 = actor_grads(*args)
    torch.cuda.synchronize()
    for k in g1:
        assert torch.equal(g1[k], g2[k])
    assert torch.equal(s1, s2)
    assert_grads(g1, r64, r32, None, F, conditioned(probs))


@pytest.mark.parametrize("F,H", [(70, 16), (30, 129), (40, 128)])  # F + 1 > 64; H > 128; H > 64 with F + 1 > 32
def test_update_rejects_bad_shapes(F, H):
    from d2dhip.update import actor_grads
    N, T, E, A = 2, 1, 8, 4
    net = {"w1": torch.zeros(N, H, F, device="cuda"), "b1": torch.zeros(N, H, device="cuda"),
           "w2": torch.zeros(N, A, H, device="cuda"), "b2": torch.zeros(N, A, device="cuda")}
    obs = torch.zeros(T, E, N, F, device="cuda")
    acts = torch.zeros(T, E, N, dtype=torch.uint8, device="cuda")
    lo = torch.zeros(T, E, N, device="cuda")
    with pytest.raises(NotImplementedError):
        actor_grads(net, obs, acts, lo, lo, "comb")


def _learner_pair(cls, kind, seed=0, E=96, N=6, H=64):
    """Two identical learners (same init, same rollout) on a small batched env.  kind "c5": the
    xp_n_agents sweep env of configs[4] (N agents, 8 channels, deadlines 7, lambda 1/14, switch 0.8)."""
    import copy
    import json
    import os
    from envs.combinatorial_env import CombinatorialEnv
    from envs.channel_selection_env import ChannelSelectionEnv
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if kind == "c5":
        params = dict(n_agents=N, n_channels=8, deadlines=np.array([7] * N), lbdas=np.full(N, 1 / 14),
                      episode_length=20, traffic_model="aperiodic", channel_switch=np.full((N, 8), 0.8))
        make_env = lambda: CombinatorialEnv(**params, n_envs=E, device="cuda", seed=seed)  # noqa: E731
    elif kind == "comb":
        cs8 = np.array(json.load(open(os.path.join(root, "d2d-ppo_amd", "combinatorial_load",
                                                   "channel_switch_8.json")))["__nd__"])
        params = dict(n_agents=N, n_channels=8, deadlines=np.array([7, 14] * 3), lbdas=np.full(N, 0.5),
                      period=np.full(N, 2), arrival_probs=np.resize(np.array([.2, .4, .8, 1, 1, 1]), N),
                      offsets=np.zeros(N), episode_length=40, traffic_model="heterogeneous",
                      homogeneous_size=False, periodic_devices=[0, 1, 2], channel_switch=np.resize(cs8, (N, 8)))
        make_env = lambda: CombinatorialEnv(**params, n_envs=E, device="cuda", seed=seed)  # noqa: E731
    else:
        params = dict(n_agents=N, n_channels=4, deadlines=np.array([7] * N), lbdas=np.full(N, 1 / 3.5),
                      period=np.full(N, 2), arrival_probs=np.full(N, 0.5), offsets=np.zeros(N),
                      episode_length=40, traffic_model="aperiodic", periodic_devices=[],
                      channel_switch=np.full(5, 0.8))
        make_env = lambda: ChannelSelectionEnv(**params, n_envs=E, device="cuda", seed=seed)  # noqa: E731
    out = []
    for _ in range(2):
        torch.manual_seed(seed)
        env = make_env()
        kw = dict(hidden_size=H, gamma=0.6, policy_lr=3e-3, value_lr=1e-3, device="cuda", useRNN=False,
                  combinatorial=kind in ("comb", "c5"))
        lr = cls(env, beta_entropy=0.05, **kw) if cls.__name__ == "D2DPPO" else cls(env, **kw)
        out.append(lr)
    torch.manual_seed(seed + 1)
    ro = out[0]._rollout(E)
    return out, ro, copy


@pytest.mark.parametrize("kind,algo,N,H", [("comb", "ippo", 6, 64), ("chsel", "ippo", 6, 64), ("comb", "d2d", 6, 64),
                                           ("chsel", "d2d", 6, 64), ("c5", "d2d", 128, 64), ("c5", "d2d", 256, 64),
                                           ("comb", "ippo", 6, 128), ("chsel", "d2d", 6, 128)])
def test_fused_epoch_matches_torch_epoch(kind, algo, N, H):
    """One learner epoch on the fused kernels == the torch agent-stacked epoch (same rollout, same
    permutation): losses 1e-5; post-Adam weights within 2% of the learning rate.  Adam's first
    steps are lr * g / (|g| + 1e-8): sign-like, so elements whose gradient is ~1e-8 move by a
    lr-sized amount that fp32-level gradient differences can change by a few 1e-3 of lr."""
    from algorithms.d2d_ppo import D2DPPO
    from algorithms.ippo import iPPO
    cls = iPPO if algo == "ippo" else D2DPPO
    (fused, ref), ro, copy = _learner_pair(cls, kind, E=96 if N <= 64 else 32, N=N, H=H)
    assert fused._fused_update_ok()
    if N > 64:  # the central critic's bf16-split GEMM path (S = 15 N + 8) is the one bench.py times
        assert ro.state_seq.shape[1] == 15 * N + 8 and fused._critic_split_forward(ro) is not None
    upd = ref._update_inputs(ro)
    for ep in range(2):
        np.random.seed(100 + ep)
        a = fused._update_epoch(ro, None)
        np.random.seed(100 + ep)
        b = ref._update_epoch(ro, upd)
        if algo == "ippo":
            assert torch.allclose(a[0], b[0], atol=1e-5), (a[0], b[0])
            assert torch.allclose(a[1], b[1], rtol=1e-5, atol=1e-5), (a[1], b[1])
        else:
            # with N > 64 the chain multiplies up to N - 1 ratios, each carrying the fp32 rounding of
            # two independent log-prob evaluations (exp(d) with |d| ~ 1e-7): the products drift by
            # ~sqrt(N) * 1e-7 relative per epoch on both paths, so later epochs get 1e-4
            tol = 1e-5 if (N <= 64 or ep == 0) else 1e-4
            print(f"  epoch {ep}: max |ploss diff| {np.abs(np.array(a[0]) - np.array(b[0])).max():.2e}  "
                  f"|vloss diff| {abs(float(a[1]) - float(b[1])):.2e}")
            assert np.allclose(a[0], b[0], atol=tol), (a[0], b[0])
            assert abs(float(a[1]) - float(b[1])) < 1e-5 * max(1.0, abs(float(b[1])))
        nets = [(fused.policy.params, ref.policy.params, 3e-3)]
        if algo == "ippo":
            nets.append((fused.value.params, ref.value.params, 1e-3))
        for pf, pr, lr in nets:
            for k in pf:
                # the (all-reduced, clipped) gradients the optimizer stepped with
                gscale = pr[k].grad.abs().max().item()
                gerr = (pf[k].grad - pr[k].grad).abs().max().item()
                err = (pf[k].data - pr[k].data).abs().max().item()
                print(f"  epoch {ep} {k}: max |g diff| / max|g| = {gerr / max(gscale, 1e-30):.2e}  "
                      f"max |w diff| / lr = {err / lr:.2e}")
                if ep == 0 or N > 64:  # both learners stepped from identical weights
                    assert gerr <= 2e-5 * gscale + 1e-9, (ep, k, gerr, gscale)
                if N <= 64:
                    assert err < 0.02 * lr, (ep, k, err)
        if N > 64:
            # c5's sparse inputs (lambda = 1/14: most buffer cells are zero in most samples) leave
            # many w1 gradients at ~1e-8, where Adam's first steps (lr * g / (|g| + 1e-8)) turn
            # fp32-level gradient differences into lr-sized weight differences; the gradients are
            # compared above, and the next epoch starts both learners from the fused one's state
            with torch.no_grad():
                for k in fused.policy.params:
                    ref.policy.params[k].copy_(fused.policy.params[k])
                for a_, b_ in zip(fused.value_network.parameters(), ref.value_network.parameters()):
                    b_.copy_(a_)
            # deep copies: load_state_dict keeps same-device state tensors by reference
            ref.policy_optimizer.load_state_dict(copy.deepcopy(fused.policy_optimizer.state_dict()))
            ref.value_optimizer.load_state_dict(copy.deepcopy(fused.value_optimizer.state_dict()))


def test_happo_chain_kernel_matches_torch_loop():
    """d2d_happo_chain == the sequential torch loop of happo_chain (d2d_ppo.py:405-433 semantics):
    ratios exp(logp_new - logp_old) and left-to-right fp32 products over the agent permutation."""
    from algorithms.d2d_ppo import happo_chain
    from d2dhip import _lib
    lib = _lib.require_gpu()
    g = torch.Generator(device="cuda").manual_seed(5)
    for N, T, E in ((1, 3, 5), (7, 20, 33), (64, 50, 128), (128, 20, 64), (256, 20, 40)):
        adv = torch.randn(T * E, device="cuda", generator=g)
        lp_old = -torch.rand((T, N, E), device="cuda", generator=g) * 3
        lp_new = lp_old.permute(1, 0, 2).reshape(N, T * E) + 0.3 * torch.randn((N, T * E), device="cuda", generator=g)
        perm = np.random.default_rng(N).permutation(N)
        ratio = torch.exp(lp_new - lp_old.permute(1, 0, 2).reshape(N, T * E))
        ref = happo_chain(adv, ratio, perm)
        M = torch.empty_like(ref)
        pt = torch.as_tensor(perm.astype(np.int32), device="cuda")
        assert lib.d2d_happo_chain(N, T, E, adv.data_ptr(), lp_new.contiguous().data_ptr(), lp_old.data_ptr(),
                                   pt.data_ptr(), M.data_ptr(), _lib.stream_ptr()) == 0
        torch.testing.assert_close(M, ref, rtol=2e-6, atol=0)


@pytest.mark.parametrize("E,agents", [(2048, None), (8192, None), (65536, (0, 21, 42, 63))],
                         ids=["2048-all", "8192-all", "65536-4agents"])
def test_grads_on_large_rollout_vs_float64(E, agents):
    """iPPO's fused actor and critic gradients on a real E-env x 200-slot rollout of the c3 config
    (64 agents x 8 channels; 409,600 / 1,638,400 samples per agent -- 8,192 envs is the longest accumulation
    chain update_blocks allows, 256 tiles per wave) against float64 autograd, EVERY agent.

    Criterion, elementwise: |g_kernel - g64| <= envelope + max(2e-5, 4 x torch fp32's own excess) x max|g64|.
    The envelope (tools/gpu/ppo_grads_full_batch.py _flip_envelope) is the largest change relu-mask flips
    can make: env observations are small integers repeated over many samples, so a layer-1 pre-activation
    within fp32 rounding of 0 (|pre| <= 2 (F + 2) u sum |w x|) may take either mask in ANY fp32 evaluation
    and flips dW1 / db1 for every sample sharing it.  The round-3 all-agent run showed such outliers of up
    to 5e-4 of max|g| in torch fp32 autograd itself (agent 27) as well as in the kernels (agents 22, 45, 59),
    each on w1 / b1 only (profiles/r03k/ppo_full_2048_all.json); the envelope is computed, not fitted,
    and is zero for every tensor but w1 / b1.  Everything outside it is held to the fp32 band.
    65,536 envs is the benched headline batch (13.1 M samples per agent; round 6: in the suite for four agents
    spread over the 64, every tensor; all 64 agents in tools/gpu/ppo_grads_full_batch.py:
    profiles/r05/ppo_full_65536_all_envelope.json)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "gpu"))
    from ppo_grads_full_batch import grads_vs_float64
    agents = range(64) if agents is None else agents
    out = grads_vs_float64(E, agents, emulate=False, envelope=True)
    checked = 0
    worst = (0.0, None)
    for key, exc in out.items():
        if not key.startswith("excess/"):
            continue
        _, net, k, n = key.split("/")
        band = max(out[f"excess32/{net}/{k}/{n}"], 0.0)
        raw = out[f"{net}/{k}/{n}"]
        if raw > 2e-5 or exc > 1e-5:
            print(f"  {net}/{k}/{n}: |kernel - f64| {raw:.2e}, outside the flip envelope {exc:.2e}, "
                  f"torch fp32 outside it {band:.2e}, ambiguous pairs {out[f'ambiguous_{net}/{k}']}")
        worst = max(worst, (exc, key))
        assert exc <= max(4 * band, 2e-5), (key, exc, band)
        checked += 1
    print(f"  worst excess over the envelope: {worst}")
    assert checked == len(agents) * 8


@pytest.mark.parametrize("H", [64, 128])
def test_deferred_values_equal_rollout_values(H):
    """iPPO training rollouts take their values from the first epoch's critic pass (d2d_ppo_critic_grad_values,
    iPPO.defer_values): the deferred rollout (_rollout(defer_values=True): actor-only slots, zero-value returns)
    on the same env draws and policy stream gives the same obs / actions / log-probs (bit-exact) and returns
    (1e-5) as the per-slot-values rollout; its first epoch's critic pass writes the same V(obs) as the rollout
    critic's forward (same weights; 1e-5), the same advantages (1e-5), and that epoch's losses (1e-5) and post-Adam
    weights (2 % of lr) equal those of the epoch on the per-slot values.  H = 64 runs the hidden-on-rows critic
    kernel, H = 128 the sample-on-rows one (its `values` write, update_kernels.hip)."""
    from algorithms.ippo import iPPO
    (ref, dfr), ro, _ = _learner_pair(iPPO, "comb", E=96, N=6, H=H)
    assert dfr._defer_values_ok()
    torch.manual_seed(1)  # _learner_pair's rollout seed: the same policy Philox stream
    ro2 = dfr._rollout(96, defer_values=True)
    assert ro2.values_pending and ro2.adv_tne is None
    assert torch.equal(ro2.obs_f32, ro.obs_f32)
    assert torch.equal(ro2.actions, ro.actions)
    assert torch.equal(ro2.logp, ro.logp)
    torch.testing.assert_close(ro2.ret_tne, ro.ret_tne, rtol=0, atol=1e-5)
    pl1, vl1 = ref._update_epoch(ro, None)
    pl2, vl2 = dfr._update_epoch(ro2, None)
    torch.testing.assert_close(ro2.values, ro.values, rtol=0, atol=1e-5)
    torch.testing.assert_close(ro2.adv_tne, ro.adv_tne, rtol=0, atol=1e-5)
    torch.testing.assert_close(pl2, pl1, rtol=0, atol=1e-5)
    torch.testing.assert_close(vl2, vl1, rtol=0, atol=1e-5)
    for net in ("policy", "value"):
        lr_ = 3e-3 if net == "policy" else 1e-3
        for k, p in getattr(ref, net).params.items():
            q = getattr(dfr, net).params[k]
            assert (p.data - q.data).abs().max().item() <= 0.02 * lr_, (net, k)
    # a second epoch on the deferred rollout runs the usual order (values are no longer pending)
    assert not ro2.values_pending
    dfr._update_epoch(ro2, None)

