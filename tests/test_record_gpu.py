"""GPU parity of the compact obs record (D2D_OBS_U8, d2dhip/record.py): the env kernel's byte rows
decode to exactly the fp32 obs it writes (combinatorial_env.py:199-206 layout), and every kernel that
reads the record -- behaviour policy (MLP and GRU), MLP actor / critic gradients, GRU gradients --
returns what it returns on the fp32 rows, bit for bit (every kernel sums in a fixed order).  Then
the learners end to end: training iterations on the record equal those on the fp32 buffer."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm GPU")
    import d2dhip
    d2dhip.require_gpu()


def comb_params(N, C, deadlines, homog, lam=0.4, switch=0.3, ep=12):
    return dict(n_agents=N, n_channels=C, deadlines=np.asarray(deadlines), lbdas=np.full(N, lam), episode_length=ep,
                traffic_model="aperiodic", homogeneous_size=homog, channel_switch=np.full((N, C), switch))


def lockstep(params, E, T, seed=11, p_act=0.3):
    """Two envs with one seed in lockstep (same actions): fp32 obs [T][E][N][F] from one, the record
    [T][E][N][R] from the other, plus the actions."""
    from envs.combinatorial_env import CombinatorialEnv
    e1 = CombinatorialEnv(**params, n_envs=E, device="cuda", seed=seed)
    e2 = CombinatorialEnv(**params, n_envs=E, device="cuda", seed=seed)
    b1, b2 = e1.batch(), e2.batch()
    s = b1.spec
    obs = torch.empty((T, E, s.N, s.F), dtype=torch.float32, device="cuda")
    rec = b2.record_buffer((T,))
    acts = torch.empty((T, E, s.N), dtype=b1.action_buffer().dtype, device="cuda")
    L = params["episode_length"]
    for t in range(T):
        if t % L == 0:
            b1.reset(out_obs=obs[t])
            b2.reset(out_obs=rec[t])
        a = b1.sample_actions(p_act)
        b2.rng_step += 1
        acts[t] = a
        if (t + 1) % L != 0 and t + 1 < T:
            b1.step(a, out_obs=obs[t + 1])
            b2.step(a, out_obs=rec[t + 1])
        else:
            b1.step(a, want_obs=False)
            b2.step(a, want_obs=False)
    return obs, rec, acts, b2


CASES = {
    "c3": (comb_params(64, 8, [7, 14] * 32, True), 70),           # the headline layout: F = 30, R = 32
    "het": (comb_params(6, 8, [7, 14, 3, 9, 14, 1], False), 33),  # per-agent widths, ACKs at moving columns
    "c16": (comb_params(8, 16, [8] * 8, True), 40),               # F = 40: two 32-input chunks, R = 64
    "wide": (comb_params(96, 32, [3, 2] * 48, False), 9),         # N > 64 (one env per workgroup), F = 67
    "c4": (comb_params(5, 4, [4, 2, 4, 2, 4], False), 17),        # ragged E
}


@pytest.mark.parametrize("case", list(CASES))
def test_env_record_decodes_to_fp32_obs(case):
    params, E = CASES[case]
    obs, rec, _, b = lockstep(params, E, 2 * params["episode_length"])
    s = b.spec
    assert torch.equal(rec.decode(), obs)
    assert bool((rec.data[..., s.F] == 1).all())                 # the bias input byte
    assert int(rec.data[..., s.F + 1:].sum()) == 0               # zero padding past it
    # values in range: counts / channel bits as uint8, acks in {-1, 0, 1}
    assert float(obs.min()) >= -1 and float(obs.max()) <= 255


def mlp_nets(N, F, H, A, seed, critic=True):
    from algorithms._core import Policy, StackedNets, Value
    torch.manual_seed(seed)
    pol = StackedNets([Policy(F, A, H) for _ in range(N)], [F] * N, "mlp", "cuda", act="softmax")
    val = StackedNets([Value(F, H) for _ in range(N)], [F] * N, "mlp", "cuda") if critic else None
    d = lambda st: {k: v.detach().contiguous() for k, v in st.params.items()}  # noqa: E731
    return d(pol), (d(val) if val is not None else None)


@pytest.mark.parametrize("case", ["c3", "het", "c16"])
@pytest.mark.parametrize("mode", ["sample", "deterministic", "forced"])
def test_policy_kernel_record_bit_exact(case, mode):
    from d2dhip.policy import policy_mlp_step
    params, E = CASES[case]
    obs, rec, acts, b = lockstep(params, E, 6)
    s = b.spec
    actor, critic = mlp_nets(s.N, s.F, 64, s.C, seed=3)
    for t in range(obs.shape[0]):
        kw = dict(rng_step=100 + t, seed=9, env_base=5, deterministic=mode == "deterministic",
                  forced=acts[t] if mode == "forced" else None)
        a1, l1, v1 = policy_mlp_step(actor, obs[t], "comb", critic, **kw)
        a2, l2, v2 = policy_mlp_step(actor, rec[t], "comb", critic, **kw)
        assert torch.equal(a1, a2) and torch.equal(l1, l2) and torch.equal(v1, v2), t


@pytest.mark.parametrize("case", ["c3", "het", "c16", "c4"])
def test_update_kernels_record_bit_exact(case):
    from d2dhip.update import actor_grads, critic_grads
    params, E = CASES[case]
    T = params["episode_length"]
    obs, rec, acts, b = lockstep(params, E, T)
    s = b.spec
    actor, critic = mlp_nets(s.N, s.F, 64, s.C, seed=4)
    g = torch.Generator(device="cuda").manual_seed(1)
    logp_old = torch.randn((T, E, s.N), device="cuda", generator=g) * 0.3 - 4.0
    adv = torch.randn((T, E, s.N), device="cuda", generator=g)
    ret = torch.randn((T, E, s.N), device="cuda", generator=g)
    ga1, sa1 = actor_grads(actor, obs, acts, logp_old, adv, "comb")
    ga1 = {k: v.clone() for k, v in ga1.items()}
    sa1 = sa1.clone()
    ga2, sa2 = actor_grads(actor, rec, acts, logp_old, adv, "comb")
    for k in ga1:
        assert torch.equal(ga1[k], ga2[k]), k
    assert torch.equal(sa1, sa2)
    gc1, sc1 = critic_grads(critic, obs, ret)
    gc1 = {k: v.clone() for k, v in gc1.items()}
    sc1 = sc1.clone()
    gc2, sc2 = critic_grads(critic, rec, ret)
    for k in gc1:
        assert torch.equal(gc1[k], gc2[k]), k
    assert torch.equal(sc1, sc2)


def gru_params(N, F, H, A, seed):
    from algorithms._core import RNN, StackedNets
    torch.manual_seed(seed)
    st = StackedNets([RNN(F, A, H) for _ in range(N)], [F] * N, "rnn", "cuda")
    # spread torch's default GRU init (uniform +-1/sqrt(H)) so the gates leave their linear regime
    return {k: (v.detach() * 3).contiguous() for k, v in st.params.items()}


@pytest.mark.parametrize("case", ["c3", "het"])
def test_gru_kernels_record(case):
    from d2dhip import gru
    params, E = CASES[case]
    L = params["episode_length"]
    obs, rec, acts, b = lockstep(params, E, 2 * L)
    s = b.spec
    p = gru_params(s.N, s.F, 32, s.C, seed=5)
    W = 5
    for slot in (0, 3, L - 1, L + 2):
        a1, l1 = gru.policy(p, obs, "sigmoid", W, L, slot, 1, rng_step=7, seed=2)
        a2, l2 = gru.policy(p, rec, "sigmoid", W, L, slot, 1, rng_step=7, seed=2)
        assert torch.equal(a1, a2) and torch.equal(l1, l2), slot
    _, lf1 = gru.policy(p, obs, "sigmoid", W, L, 0, 2 * L, padded=True, forced=acts)
    _, lf2 = gru.policy(p, rec, "sigmoid", W, L, 0, 2 * L, padded=True, forced=acts)
    assert torch.equal(lf1, lf2)
    g = torch.Generator(device="cuda").manual_seed(2)
    adv = torch.randn((2 * L, E, s.N), device="cuda", generator=g)
    g1, st1 = gru.grads(p, obs, "sigmoid", W, L, adv, actions=acts, logp_old=lf1.view(s.N, 2 * L, E).permute(1, 2, 0))
    g1 = {k: v.clone() for k, v in g1.items()}
    st1 = st1.clone()
    g2, st2 = gru.grads(p, rec, "sigmoid", W, L, adv, actions=acts, logp_old=lf1.view(s.N, 2 * L, E).permute(1, 2, 0))
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k
    assert torch.equal(st1, st2)
    # and the GRU gradients are reproducible run to run (fixed-order sums, no atomics)
    g3, st3 = gru.grads(p, rec, "sigmoid", W, L, adv, actions=acts, logp_old=lf1.view(s.N, 2 * L, E).permute(1, 2, 0))
    for k in g1:
        assert torch.equal(g1[k], g3[k]), k


@pytest.mark.parametrize("rnn", [False, True])
@pytest.mark.parametrize("algo", ["ippo", "d2d"])
def test_learner_iteration_on_record_equals_fp32(algo, rnn):
    """Training iterations (rollout, GAE, epochs of fused updates) on the record give the same
    parameters as on the fp32 buffer, bit for bit."""
    from algorithms.d2d_ppo import D2DPPO
    from algorithms.ippo import iPPO
    from envs.combinatorial_env import CombinatorialEnv
    out = []
    for use_rec in (False, True):
        torch.manual_seed(0)
        np.random.seed(0)
        env = CombinatorialEnv(**comb_params(6, 8, [7, 14] * 3, True, ep=20), n_envs=48, device="cuda", seed=3)
        common = dict(hidden_size=32, gamma=0.5, device="cuda", combinatorial=True, early_stopping=False,
                      useRNN=rnn, history_len=4)
        lr = iPPO(env, **common) if algo == "ippo" else D2DPPO(env, **common)
        lr.obs_record = use_rec
        lr.train(num_iter=2, n_epoch=2, num_episodes=48, test_freq=100)
        from d2dhip.record import ObsRecord
        ro = lr._rollout(48)
        assert isinstance(ro.obs, ObsRecord) == use_rec
        out.append([v.detach().clone() for v in lr.policy.params.values()])
    for a, b in zip(*out):
        assert torch.equal(a, b)
