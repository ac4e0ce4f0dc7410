"""GPU parity of the D2DEnv kernel (csrc/env_kernels.hip single_kernel; pytest -m gpu).

1. replay: the reference D2DEnv's recorded actions / channel flips / arrivals
   (tests/golden/d2denv_*.npz, tools/gen_fixtures.py gen_d2denv) through the
   HIP kernel give the reference's obs, state, ACK, rewards, buffers, channel
   states and counters bit for bit, for E = 3 copies of each trace;
2. Philox production mode == the numpy oracle (oracle/env_oracle.py "single")
   bit for bit, incl. N > 64 (one env per workgroup) and full neighbourhoods;
3. the reference-API path (n_envs = 1 numpy structures, counters);
4. the learners run on it (iPPO and D2D-PPO, one iteration + test());
5. the compact obs record (ABI 14) decodes to the fp32 obs bit for bit.
Bit-exact for every integer output; obs / state exact after the fp32 cast.
"""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_params

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm GPU")
    import d2dhip
    d2dhip.require_gpu()


def fixtures():
    return sorted(os.path.basename(p)[7:-4] for p in glob.glob(os.path.join(GOLDEN, "d2denv_*.npz")))


def make(params, **kw):
    from envs.env import D2DEnv
    p = {k: v for k, v in params.items() if k != "verbose"}
    return D2DEnv(**p, **kw)


@pytest.mark.parametrize("name", fixtures())
def test_replay_matches_reference(name):
    z = np.load(os.path.join(GOLDEN, f"d2denv_{name}.npz"))
    params = load_params(z)
    E = 3
    env = make(params, n_envs=E, device="cuda", seed=1)
    b = env.batch()
    s = b.spec
    dev = b.device
    L = int(params["episode_length"])
    rep = lambda a: np.repeat(np.asarray(a)[None], E, axis=0)  # noqa: E731
    W = z["obs"].shape[2]
    step = 0
    for ep in range(int(z["episodes"])):
        arr0 = torch.from_numpy(rep(z["reset_arrivals"][ep]).astype(np.uint8)).to(dev)
        r = env.reset_batched(want_obs=True, want_state=True, replay_arrivals=arr0)
        obs = r["obs"].cpu().numpy()
        st = r["state"].cpu().numpy()[:, : s.S]
        for e in range(E):
            assert np.array_equal(obs[e, :, :W], z["reset_obs"][ep]), (ep, e)
            assert not obs[e, :, W:].any()
            assert np.array_equal(st[e], z["reset_state"][ep]), (ep, e)
        assert np.array_equal(b.channels_host(), rep(z["reset_chan"][ep]))
        for t in range(L):
            act = torch.from_numpy(rep(z["actions"][step]).astype(np.uint8)).to(dev)
            fl = torch.from_numpy(rep(z["flips"][step]).astype(np.uint8)).to(dev)
            arr = torch.from_numpy(rep(z["arrivals"][step]).astype(np.uint8)).to(dev)
            out = env.step_batched(act, want_obs=True, want_state=True, want_ack=True, want_success=True,
                                   replay=(fl, arr))
            obs = out["obs"].cpu().numpy()
            st = out["state"].cpu().numpy()[:, : s.S]
            for e in range(E):
                assert np.array_equal(obs[e, :, :W], z["obs"][step]), (ep, t, e)
                assert np.array_equal(st[e], z["state"][step]), (ep, t, e)
            assert np.all(out["ack"].cpu().numpy() == z["ack"][step])
            assert np.all(out["reward"].cpu().numpy() == z["rewards"][step][0])
            assert np.array_equal(out["success"].cpu().numpy().astype(bool), rep(z["success"][step]))
            assert np.array_equal(b.buffers_host(), rep(z["buffers"][step]))
            assert np.array_equal(b.channels_host(), rep(z["chan"][step]))
            assert np.array_equal(b.received.cpu().numpy(), rep(z["received"][step]))
            assert np.array_equal(b.discarded.cpu().numpy(), rep(z["discarded"][step]))
            assert np.all(b.sel_quality.cpu().numpy() == z["channel_errors"][step])
            assert np.all(b.sel_count.cpu().numpy() == z["n_collisions"][step])
            assert out["done"] == bool(z["done"][step])
            step += 1


# ------------------------------------------------------------ Philox vs oracle
def _philox_case(params, E, steps, seed, episodes=2, p_act=0.3):
    from oracle import philox
    from oracle.env_oracle import EnvOracle
    env = make(params, n_envs=E, device="cuda", seed=seed)
    b = env.batch()
    s = b.spec
    o = EnvOracle("single", params, n_envs=E, seed=seed)
    envs = np.arange(E, dtype=np.uint64)
    for ep in range(episodes):
        r = env.reset_batched(want_obs=True, want_state=True)
        ro = o.reset(rng_step=b.rng_step - 1)
        assert np.array_equal(r["obs"].cpu().numpy(), ro["obs"].astype(np.float32)), ep
        assert np.array_equal(r["state"].cpu().numpy()[:, : s.S], ro["state"].astype(np.float32)), ep
        for t in range(steps):
            rs = b.rng_step
            a = b.sample_actions(p_act)
            w = philox.words(envs[:, None], np.arange(s.N, dtype=np.uint64)[None, :], rs, philox.STREAM_ACTION, 1,
                             seed)[..., 0]
            ac = (w < philox.threshold(p_act)).astype(np.int64)       # GFAccess-style Bernoulli(p) attempts
            assert np.array_equal(a.cpu().numpy(), ac), (ep, t)
            rs = b.rng_step
            out = env.step_batched(a, want_obs=True, want_state=True, want_ack=True, want_success=True)
            oc = o.step(ac, rng_step=rs)
            assert np.array_equal(out["obs"].cpu().numpy(), oc["obs"].astype(np.float32)), (ep, t)
            assert np.array_equal(out["state"].cpu().numpy()[:, : s.S], oc["state"].astype(np.float32)), (ep, t)
            assert np.array_equal(out["reward"].cpu().numpy(), oc["rewards"].astype(np.int32)), (ep, t)
            assert np.array_equal(out["ack"].cpu().numpy(), oc["ack"][:, 0].astype(np.int8)), (ep, t)
            assert np.array_equal(out["success"].cpu().numpy().astype(bool), oc["success"]), (ep, t)
            assert np.array_equal(b.buffers_host(), o.buffers), (ep, t)
            assert np.array_equal(b.channels_host(), o.chan), (ep, t)
            assert np.array_equal(b.received.cpu().numpy(), o.received)
            assert np.array_equal(b.discarded.cpu().numpy(), o.discarded)
            assert np.array_equal(b.sel_quality.cpu().numpy(), o.channel_errors)
            assert np.array_equal(b.sel_count.cpu().numpy(), o.n_collisions)


@pytest.mark.parametrize("name", fixtures())
def test_philox_matches_oracle(name):
    z = np.load(os.path.join(GOLDEN, f"d2denv_{name}.npz"))
    params = load_params(z)
    params["episode_length"] = 12
    _philox_case(params, E=129, steps=12, seed=20261016)


@pytest.mark.parametrize("N,full", [(65, False), (96, True), (200, False), (1024, False)])
def test_philox_large_agent_counts(N, full):
    """N > 64: one env per workgroup, LDS-accumulated attempt counts; full neighbourhoods
    make obs rows N*(d+1)+1 long (gathered from the env's rows staged in LDS)."""
    d = np.array([3, 5, 7] * (N // 3) + [4] * (N % 3))
    nb = [list(range(N)) for _ in range(N)] if full else [[(k - 1) % N, k, (k + 1) % N] for k in range(N)]
    params = dict(n_agents=N, deadlines=d, lbdas=np.full(N, 0.05), episode_length=8, channel_switch=0.3,
                  neighbourhoods=nb)
    _philox_case(params, E=5, steps=8, seed=7, p_act=0.02)


def _record_case(params, E, steps, seed, p_act=0.05):
    """Two identical batches, one emitting fp32 obs rows and one the compact record (ABI 14): the decoded record is
    the fp32 obs bit for bit at every reset and step, and the env states stay identical."""
    from envs.env import D2DEnv  # noqa: F401
    envs = [make(params, n_envs=E, device="cuda", seed=seed) for _ in range(2)]
    ba, bb = envs[0].batch(), envs[1].batch()
    rec = bb.record_buffer(())
    L = int(params["episode_length"])
    act = ba.action_buffer()
    for t in range(steps):
        if t % L == 0:
            ra = ba.reset(want_obs=True)
            bb.reset(want_obs=True, out_obs=rec)
            assert torch.equal(rec.decode(), ra["obs"]), ("reset", t)
        ba.sample_actions(p_act, out=act)
        bb.rng_step += 1  # (the sampler's draw on the other batch)
        ra = ba.step(act, want_obs=True)
        bb.step(act, out_obs=rec)
        torch.cuda.synchronize()
        assert torch.equal(rec.decode(), ra["obs"]), t
        for x, y in ((ba.buffers, bb.buffers), (ba.channels, bb.channels), (ba.received, bb.received),
                     (ba.discarded, bb.discarded), (ba.reward, bb.reward)):
            assert torch.equal(x, y), t
    # the row's bias byte (column F) and zeros past it
    R = rec.data.shape[-1]
    F = ba.spec.F
    assert torch.all(rec.data[..., F] == 1) and (R == F + 1 or torch.all(rec.data[..., F + 1:] == 0))


@pytest.mark.parametrize("name", fixtures())
def test_record_equals_fp32_obs(name):
    """The D2DEnv compact record (single_kernel, ABI 14): 32 bytes per agent-step for the learners instead of 4 F of
    fp32 rows, decoded bit-exactly to the obs the reference's env.py:89-95 layout gives (the fp32 rows are pinned to
    the reference traces by test_replay_matches_reference)."""
    z = np.load(os.path.join(GOLDEN, f"d2denv_{name}.npz"))
    params = load_params(z)
    params["episode_length"] = 7
    _record_case(params, E=133, steps=15, seed=99)


@pytest.mark.parametrize("N", [64, 65, 200])
def test_record_ring_agent_counts(N):
    d = np.array([3, 5, 7] * (N // 3) + [4] * (N % 3))
    nb = [[(k - 1) % N, k, (k + 1) % N] for k in range(N)]
    params = dict(n_agents=N, deadlines=d, lbdas=np.full(N, 0.1), episode_length=6, channel_switch=0.3,
                  neighbourhoods=nb)
    _record_case(params, E=37 if N > 64 else 1001, steps=13, seed=5, p_act=0.1)


def test_record_too_wide_is_refused():
    """Full neighbourhoods of 96 agents: the record's gather codes do not fit the workgroup's LDS -- refused loudly
    (the learners keep fp32 rows there: _record_ok)."""
    N = 96
    params = dict(n_agents=N, deadlines=np.full(N, 7), lbdas=np.full(N, 0.1), episode_length=6, channel_switch=0.3,
                  neighbourhoods=[list(range(N)) for _ in range(N)])
    env = make(params, n_envs=4, device="cuda", seed=1)
    b = env.batch()
    rec = b.record_buffer(())
    with pytest.raises(NotImplementedError, match="LDS"):
        b.reset(want_obs=True, out_obs=rec)


def test_reference_api_structures():
    """n_envs = 1: reset -> (obs list, state array); step -> (obs, state, float rewards = ack, done, {});
    counters and metrics as the reference attributes (env.py:80-99, 197-213)."""
    from oracle.env_oracle import EnvOracle
    z = np.load(os.path.join(GOLDEN, "d2denv_6_full_nbr.npz"))
    params = load_params(z)
    params["episode_length"] = 20
    env = make(params, n_envs=1, device="cuda", seed=11)
    o = EnvOracle("single", params, n_envs=1, seed=11)
    obs, state = env.reset()
    ro = o.reset(rng_step=0)
    assert isinstance(obs, list) and len(obs) == env.n_agents
    for k in range(env.n_agents):
        assert obs[k].dtype == np.float64 and obs[k].shape == env.observation_space[k].shape
        assert np.array_equal(obs[k], ro["obs"][0, k, : obs[k].shape[0]])
    assert state.shape == env.state_space.shape and np.array_equal(state, ro["state"][0])
    rng = np.random.default_rng(3)
    tot_succ = 0
    for t in range(20):
        a = (rng.random(env.n_agents) < 0.35).astype(np.int64)
        obs, state, rewards, done, info = env.step(a)
        oc = o.step(a[None], rng_step=t + 1)
        assert rewards.dtype == np.float64 and rewards.shape == (env.n_agents,)
        assert np.all(rewards == oc["rewards"][0]) and info == {}
        assert env.last_feedback == oc["ack"][0, 0]
        for k in range(env.n_agents):
            assert np.array_equal(obs[k], oc["obs"][0, k, : obs[k].shape[0]])
        assert np.array_equal(state, oc["state"][0])
        assert env.channel_errors == o.channel_errors[0] and env.n_collisions == o.n_collisions[0]
        assert np.array_equal(env.channel_state, o.chan[0].astype(np.float64))
        tot_succ += int(oc["ack"][0, 0] == 1)
        assert done == (t + 1 >= 20)
    assert env.successful_transmissions == tot_succ == o.successful_transmissions[0]
    assert np.isclose(env.compute_jains(), o.compute_jains()[0], rtol=0, atol=1e-15)
    assert np.isclose(env.compute_urllc(), o.compute_urllc()[0], rtol=0, atol=1e-15)
    with pytest.raises(ValueError, match="0 or 1"):
        env.step(np.full(env.n_agents, 2))


@pytest.mark.parametrize("algo", ["ippo", "d2d"])
def test_learners_run_on_d2denv(algo):
    """iPPO / D2D-PPO on the D2DEnv (Discrete(2) actions, neighbourhood observations of unequal
    lengths): one training iteration and a test() pass, channel errors counted per episode."""
    from algorithms.d2d_ppo import D2DPPO
    from algorithms.ippo import iPPO
    N = 6
    nb = [[k, (k + 1) % N] for k in range(N - 1)] + [[N - 1]]
    env = make(dict(n_agents=N, deadlines=np.array([3, 5] * 3), lbdas=np.full(N, 0.3), episode_length=25,
                    neighbourhoods=nb), n_envs=64, device="cuda", seed=5)
    common = dict(hidden_size=32, gamma=0.9, policy_lr=3e-3, value_lr=1e-2, device="cuda", early_stopping=False)
    lr = iPPO(env, **common) if algo == "ippo" else D2DPPO(env, beta_entropy=0.02, **common)
    w0 = [p.detach().clone() for p in lr.policy.parameters()]
    lr.train(1, n_epoch=2, num_episodes=64, test_freq=1000)
    assert any(not torch.equal(a, p.detach()) for a, p in zip(w0, lr.policy.parameters()))
    score, jains, ch, rew = lr.test(64)
    assert 0.0 <= score <= 1.0 and 0.0 < jains <= 1.0 + 1e-12
    assert ch >= 0 and float(ch) == int(ch)
    assert -25.0 <= rew <= 25.0
