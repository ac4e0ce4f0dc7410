"""GPU parity of the fused behaviour-policy kernel (csrc/policy_kernels.hip) against a
plain torch fp32 reference of the same op (the reference's Policy/Value forward +
torch.distributions Bernoulli/Categorical, algorithms/ippo.py:54-90,154-176), with the
reference's initialisation (orthogonal, gain 2) and env-like observations.
Tolerance: values 1e-5 absolute; log-probs 1e-5 absolute wherever every probability of
the (agent, env) lies in [1e-3, 1-1e-3]; elsewhere log(1-p) for p -> 1 is ill-conditioned
in fp32 for BOTH implementations (a 1-ulp difference in p is a relative 6e-8/(1-p)
difference in 1-p), so there 1e-3.  Actions exact (sampled actions are compared with the
same Philox uniforms, ties |u - p| < 1e-6 excluded).
Both kernels are covered: the default exact-split bf16 MFMA kernel and the fp32-MFMA one
(D2D_OPT_POLICY_F32_MFMA); fractional observations exercise the split kernel's six-term path."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(params=["split", "f32"], autouse=True)
def impl(request):
    from d2dhip import _lib
    lib = _lib.require_gpu()
    lib.d2d_set_option(_lib.D2D_OPT_POLICY_F32_MFMA, 1 if request.param == "f32" else 0)
    yield request.param
    lib.d2d_set_option(_lib.D2D_OPT_POLICY_F32_MFMA, 0)


def make(kind, N, E, F, H, A, in_dims=None, seed=0, critic=True, frac=False):
    from algorithms._core import Policy, StackedNets, Value
    torch.manual_seed(seed)
    dims = in_dims or [F] * N
    pol = StackedNets([Policy(d, A, H) for d in dims], dims, "mlp", "cpu", act="softmax")
    val = StackedNets([Value(d, H) for d in dims], dims, "mlp", "cpu") if critic else None
    g = torch.Generator().manual_seed(seed + 1)
    obs = torch.zeros(E, N, F)
    D = F // 3
    obs[:, :, :D] = torch.randint(0, 3, (E, N, D), generator=g).float()            # buffer counts
    obs[:, :, D:] = torch.randint(-1, 2, (E, N, F - D), generator=g).float()       # channel bits / ACK
    if frac:  # values that are not bf16-exact
        obs += torch.rand(obs.shape, generator=g) * 0.3
    for k, d in enumerate(dims):
        obs[:, k, d:] = 0
    dev = "cuda"
    to = lambda st: None if st is None else {k: v.detach().to(dev).contiguous() for k, v in st.params.items()}  # noqa
    return to(pol), to(val), obs.to(dev)


def torch_ref(actor, crit, obs):
    x = obs.transpose(0, 1)  # [N][E][F]
    h = torch.relu(torch.baddbmm(actor["b1"].unsqueeze(1), x, actor["w1"].transpose(1, 2)))
    probs = torch.softmax(torch.baddbmm(actor["b2"].unsqueeze(1), h, actor["w2"].transpose(1, 2)), -1)
    v = None
    if crit is not None:
        hv = torch.relu(torch.baddbmm(crit["b1"].unsqueeze(1), x, crit["w1"].transpose(1, 2)))
        v = torch.baddbmm(crit["b2"].unsqueeze(1), hv, crit["w2"].transpose(1, 2))[..., 0]
    return probs, v


CASES = [("comb", 30, 64, 8, None), ("comb", 30, 64, 8, [23, 30, 23, 30, 23, 30, 30]), ("comb", 46, 64, 16, None),
         ("comb", 10, 20, 3, None), ("chsel", 12, 16, 5, None), ("chsel", 24, 64, 16, [24, 20, 24, 21, 24, 24, 24]),
         ("chsel", 8, 40, 2, None), ("comb", 63, 32, 8, None), ("comb", 64, 64, 8, None), ("chsel", 31, 48, 9, None),
         # the learners' default hidden_size 128 (ippo.py:225, d2d_ppo.py:222) and the modules' default 100
         ("comb", 30, 128, 8, None), ("chsel", 12, 128, 5, None), ("comb", 23, 100, 8, [23, 20, 23, 23, 23, 23, 23])]


@pytest.mark.parametrize("frac", [False, True])
@pytest.mark.parametrize("kind,F,H,A,in_dims", CASES)
def test_forced_and_deterministic_match_torch(kind, F, H, A, in_dims, frac):
    from d2dhip.envbatch import pack_masks_torch
    from d2dhip.policy import policy_mlp_step
    from torch.distributions import Bernoulli, Categorical
    N, E = 7, 301
    actor, crit, obs = make(kind, N, E, F, H, A, in_dims, frac=frac)
    probs, v = torch_ref(actor, crit, obs)
    g = torch.Generator(device="cuda").manual_seed(3)
    if kind == "comb":
        bits = (torch.rand((N, E, A), device="cuda", generator=g) < 0.4).float()
        forced = pack_masks_torch(bits.transpose(0, 1))
        ref_lp = Bernoulli(probs=probs, validate_args=False).log_prob(bits).mean(-1)
    else:
        ids = torch.randint(0, A, (N, E), device="cuda", generator=g)
        forced = ids.t().to(torch.uint8).contiguous()
        ref_lp = Categorical(probs=probs, validate_args=False).log_prob(ids)
    acts, lp, val = policy_mlp_step(actor, obs, kind, crit, forced=forced)
    assert torch.equal(acts, forced)
    well = ((probs > 1e-3) & (probs < 1 - 1e-3)).all(-1)
    torch.testing.assert_close(lp[well], ref_lp[well], rtol=0, atol=1e-5)
    torch.testing.assert_close(lp, ref_lp, rtol=0, atol=1e-3)
    torch.testing.assert_close(val, v, rtol=0, atol=1e-5)
    # deterministic evaluation actions (ippo.py:166 / 171)
    acts_d, lp_d, _ = policy_mlp_step(actor, obs, kind, None, deterministic=True)
    if kind == "comb":
        want = pack_masks_torch((probs > 0.5).transpose(0, 1))
    else:
        want = probs.argmax(-1).t().to(torch.uint8)
    assert torch.equal(acts_d, want)


@pytest.mark.parametrize("N", [128, 256])
def test_c5_agent_counts_match_torch(N):
    """configs[4] shapes (xp_n_agents sweep at 128 / 256 agents, C = 8, D = 7 -> F = 23, H = 64):
    forced log-probs 1e-5 where well conditioned, deterministic actions exact."""
    from d2dhip.envbatch import pack_masks_torch
    from d2dhip.policy import policy_mlp_step
    from torch.distributions import Bernoulli
    E, F, H, A = 520, 23, 64, 8
    actor, _, obs = make("comb", N, E, F, H, A, seed=N, critic=False)
    probs, _ = torch_ref(actor, None, obs)
    g = torch.Generator(device="cuda").manual_seed(N)
    bits = (torch.rand((N, E, A), device="cuda", generator=g) < 0.3).float()
    forced = pack_masks_torch(bits.transpose(0, 1))
    ref_lp = Bernoulli(probs=probs, validate_args=False).log_prob(bits).mean(-1)
    acts, lp, _ = policy_mlp_step(actor, obs, "comb", None, forced=forced)
    assert torch.equal(acts, forced)
    well = ((probs > 1e-3) & (probs < 1 - 1e-3)).all(-1)
    assert well.float().mean() > 0.5
    torch.testing.assert_close(lp[well], ref_lp[well], rtol=0, atol=1e-5)
    acts_d, _, _ = policy_mlp_step(actor, obs, "comb", None, deterministic=True)
    assert torch.equal(acts_d, pack_masks_torch((probs > 0.5).transpose(0, 1)))


@pytest.mark.parametrize("kind,F,H,A,in_dims", CASES[:1] + CASES[4:5])
def test_sampling_uses_philox_stream3(kind, F, H, A, in_dims):
    import sys, os
    from oracle import philox
    from d2dhip.policy import policy_mlp_step
    N, E = 5, 200
    actor, crit, obs = make(kind, N, E, F, H, A, in_dims, seed=9)
    probs, _ = torch_ref(actor, crit, obs)
    p = probs.double().cpu().numpy()                                   # [N][E][A]
    seed, base, step = 1234, 77, 5
    acts, lp, _ = policy_mlp_step(actor, obs, kind, None, rng_step=step, seed=seed, env_base=base)
    envs = (base + np.arange(E)).astype(np.uint64)
    agents = np.arange(N, dtype=np.uint64)
    if kind == "comb":
        r = philox.words(envs[None, :], agents[:, None], step, 3, 4 * ((A + 3) // 4), seed)  # [N][E][4*blk]
        u = (r[..., :A] >> np.uint64(8)).astype(np.float64) / 16777216.0
        bits = (u < p).astype(np.uint8)
        got = np.unpackbits(acts.cpu().numpy().view(np.uint8).reshape(E, N, -1), axis=2, bitorder="little")[:, :, :A]
        near = np.abs(u - p) < 1e-6
        assert np.array_equal(np.where(near, 0, got.transpose(1, 0, 2)), np.where(near, 0, bits))
        assert abs(got.mean() - p.mean()) < 0.05
    else:
        r = philox.words(envs[None, :], agents[:, None], step, 3, 1, seed)[..., 0]
        u = (r >> np.uint64(8)).astype(np.float64) / 16777216.0
        cdf = np.cumsum(p, -1)
        want = np.minimum((u[..., None] * cdf[..., -1:] >= cdf).sum(-1), A - 1)
        got = acts.cpu().numpy().T
        assert (got == want).mean() > 0.995
    # the log-prob returned with a sample equals the forced evaluation of that sample
    _, lp2, _ = policy_mlp_step(actor, obs, kind, None, forced=acts)
    torch.testing.assert_close(lp, lp2, rtol=0, atol=0)


@pytest.mark.parametrize("kind,F,H,A,in_dims", [CASES[0], CASES[4], CASES[3], CASES[2]])
def test_forced_full_waves_equal_sampled_logp(kind, F, H, A, in_dims):
    """Batches large enough for many tiles per wave (one resident round: the forced bytes travel through the
    obs DMA ring, several hundred tile pairs per wave) with a ragged tail: the forced evaluation of sampled actions
    reproduces their log-probs bit for bit (the D2D first-epoch identity), and matches torch (1e-5,
    well-conditioned)."""
    from torch.distributions import Bernoulli, Categorical
    from d2dhip.policy import policy_mlp_step
    from d2dhip.envbatch import pack_masks_torch
    N, E = 8, 65536 + 1000 + 7
    actor, _, obs = make(kind, N, E, F, H, A, in_dims, seed=4, critic=False)
    acts, lp, _ = policy_mlp_step(actor, obs, kind, None, rng_step=2, seed=99)
    acts2, lp2, _ = policy_mlp_step(actor, obs, kind, None, forced=acts)
    assert torch.equal(acts2, acts)
    torch.testing.assert_close(lp2, lp, rtol=0, atol=0)
    # ABI 15: the same log-probs with actions = NULL (D2D-PPO's epoch-start pass; A > 8 and the Categorical ids
    # through the epilogue's own load, A <= 8 through the DMA ring)
    none3, lp3, _ = policy_mlp_step(actor, obs, kind, None, forced=acts, want_actions=False)
    assert none3 is None
    torch.testing.assert_close(lp3, lp, rtol=0, atol=0)
    probs, _ = torch_ref(actor, None, obs)
    if kind == "comb":
        bits = torch.stack([(acts.long() >> j) & 1 for j in range(A)], -1).transpose(0, 1).float()  # [N][E][A]
        assert torch.equal(pack_masks_torch(bits.transpose(0, 1)), acts)
        ref_lp = Bernoulli(probs=probs, validate_args=False).log_prob(bits).mean(-1)
    else:
        ref_lp = Categorical(probs=probs, validate_args=False).log_prob(acts.t().long())
    well = ((probs > 1e-3) & (probs < 1 - 1e-3)).all(-1)
    torch.testing.assert_close(lp2[well], ref_lp[well], rtol=0, atol=1e-5)


@pytest.mark.parametrize("kind,F,H,A", [("comb", 30, 64, 8), ("chsel", 12, 64, 5)])
def test_one_round_waves_and_critic_split(kind, F, H, A):
    """Sampling, deterministic and forced launches all size every wave to one resident round (64 agents x 32,845
    envs: about 1,000 envs per wave, a ragged tail; the forced bytes travel through the obs DMA ring).  The sampled
    log-probs equal the forced evaluation's bit for bit, values match torch (1e-5), and the actor + value-only
    launches (D2D_OPT_POLICY_CRITIC_SPLIT) reproduce the fused kernel's actions, log-probs and values bit for bit --
    also with critic weights and value = NULL (the value-only launch is skipped, nothing is stored)."""
    from d2dhip import _lib
    from d2dhip.policy import policy_mlp_step
    lib = _lib.require_gpu()
    N, E = 64, 32768 + 77
    actor, crit, obs = make(kind, N, E, F, H, A, seed=11)
    acts, lp, val = policy_mlp_step(actor, obs, kind, crit, rng_step=4, seed=5)
    acts2, lp2, val2 = policy_mlp_step(actor, obs, kind, crit, forced=acts)
    assert torch.equal(acts2, acts)
    torch.testing.assert_close(lp2, lp, rtol=0, atol=0)
    torch.testing.assert_close(val2, val, rtol=0, atol=0)
    _, v = torch_ref(actor, crit, obs)
    torch.testing.assert_close(val, v, rtol=0, atol=1e-5)
    try:
        lib.d2d_set_option(_lib.D2D_OPT_POLICY_CRITIC_SPLIT, 1)
        acts3, lp3, val3 = policy_mlp_step(actor, obs, kind, crit, rng_step=4, seed=5)
        acts_d3, lp_d3, val_d3 = policy_mlp_step(actor, obs, kind, crit, deterministic=True)
        acts4, lp4, val4 = policy_mlp_step(actor, obs, kind, crit, rng_step=4, seed=5, want_value=False)
        torch.cuda.synchronize()
    finally:
        lib.d2d_set_option(_lib.D2D_OPT_POLICY_CRITIC_SPLIT, 0)
    assert torch.equal(acts3, acts)
    torch.testing.assert_close(lp3, lp, rtol=0, atol=0)
    assert val4 is None and torch.equal(acts4, acts)
    torch.testing.assert_close(lp4, lp, rtol=0, atol=0)
    torch.testing.assert_close(val3, val, rtol=0, atol=0)
    acts_d, lp_d, val_d = policy_mlp_step(actor, obs, kind, crit, deterministic=True)
    assert torch.equal(acts_d3, acts_d)
    torch.testing.assert_close(lp_d3, lp_d, rtol=0, atol=0)
    torch.testing.assert_close(val_d3, val_d, rtol=0, atol=0)
