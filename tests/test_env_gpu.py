"""GPU parity of the HIP env kernels (run on the MI355X box: pytest -m gpu).

1. replay: the reference's recorded draws through the HIP kernels must give
   the reference's outputs bit for bit (every golden fixture, E envs at once);
2. Philox production mode: HIP == C oracle bit for bit (obs, state, rewards,
   ACK, success, buffers, channels, counters), incl. N > 64 (multi-wave envs);
3. the reference-API path (n_envs=1 numpy structures) == C oracle;
4. full size (64 x 8 x 65536): bit-exact vs the C oracle for a few slots, and
   size-independent invariants over a whole episode.
Bit-exact for every integer/mask output; obs/state exact after the fp32 cast.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, env_fixture_names, load_params

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm GPU")
    import d2dhip
    d2dhip.require_gpu()


def make_env(kind, params, **kw):
    from envs.channel_selection_env import ChannelSelectionEnv
    from envs.combinatorial_env import CombinatorialEnv
    cls = CombinatorialEnv if kind == "comb" else ChannelSelectionEnv
    p = dict(params)
    if kind == "chsel":
        p.pop("homogeneous_size", None)
        p.pop("collision_type", None)
    return cls(**p, **kw)


def pack(bits, C):
    from d2dhip.envbatch import pack_masks
    return pack_masks(bits, C)


def chsel_flip_words(f):
    f = np.asarray(f, dtype=np.int64)
    return (f << np.arange(f.shape[-1])).sum(-1).astype(np.int32)


# ------------------------------------------------------------------ replay
@pytest.mark.parametrize("name", env_fixture_names())
def test_replay_matches_reference(name):
    z = np.load(os.path.join(GOLDEN, f"env_{name}.npz"))
    kind = str(z["kind"])
    params = load_params(z)
    E = 3
    env = make_env(kind, params, n_envs=E, device="cuda", seed=1)
    b = env.batch()
    s = b.spec
    dev = b.device
    L = int(params["episode_length"])
    rep = lambda a: np.repeat(np.asarray(a)[None], E, axis=0)  # noqa: E731
    step = 0
    for ep in range(int(z["episodes"])):
        arr0 = torch.from_numpy(rep(z["reset_arrivals"][ep]).astype(np.uint8)).to(dev)
        r = env.reset_batched(want_obs=True, want_state=True, replay_arrivals=arr0)
        torch.cuda.synchronize()
        obs = r["obs"].cpu().numpy()
        st = r["state"].cpu().numpy()[:, : s.S]
        for e in range(E):
            assert np.array_equal(obs[e], z["reset_obs"][ep].astype(np.float32)), (ep, e)
            assert np.array_equal(st[e], z["reset_state"][ep].astype(np.float32)), (ep, e)
        for t in range(L):
            if kind == "comb":
                act = torch.from_numpy(pack(rep(z["actions"][step]), s.C)).to(dev)
                fl = torch.from_numpy(pack(rep(z["flips"][step]), s.C)).to(dev)
            else:
                act = torch.from_numpy(rep(z["actions"][step]).astype(np.uint8)).to(dev)
                fl = torch.from_numpy(rep(chsel_flip_words(z["flips"][step]))).to(dev)
            arr = torch.from_numpy(rep(z["arrivals"][step]).astype(np.uint8)).to(dev)
            out = env.step_batched(act, want_obs=True, want_state=True, want_ack=True, want_success=True,
                                   replay=(fl, arr))
            obs = out["obs"].cpu().numpy()
            st = out["state"].cpu().numpy()[:, : s.S]
            ack = out["ack"].cpu().numpy()
            rew = out["reward"].cpu().numpy()
            succ = out["success"].cpu().numpy()
            bufs = b.buffers_host()
            chans = b.channels_host()
            recv = b.received.cpu().numpy()
            disc = b.discarded.cpu().numpy()
            for e in range(E):
                assert np.array_equal(obs[e], z["obs"][step].astype(np.float32)), (ep, t, e)
                assert np.array_equal(st[e], z["state"][step].astype(np.float32)), (ep, t, e)
                assert np.array_equal(ack[e], z["ack"][step].astype(ack.dtype)), (ep, t, e)
                assert rew[e] == z["rewards"][step][0]
                assert np.array_equal(succ[e].astype(bool), z["success"][step])
                assert np.array_equal(bufs[e], z["buffers"][step])
                assert np.array_equal(chans[e], z["chan"][step])
                assert np.array_equal(recv[e], z["received"][step]) and np.array_equal(disc[e], z["discarded"][step])
            if kind == "chsel":
                assert np.all(b.sel_quality.cpu().numpy() == z["sel_q"][step])
                assert np.all(b.sel_count.cpu().numpy() == z["sel_n"][step])
            assert out["done"] == bool(z["done"][step])
            step += 1


# ---------------------------------------------------------- Philox vs C oracle
def _philox_case(kind, params, E, steps, seed, episodes=2, p_act=0.25):
    from oracle.c_oracle import COracle
    env = make_env(kind, params, n_envs=E, device="cuda", seed=seed)
    b = env.batch()
    s = b.spec
    c = COracle(kind, params, n_envs=E, seed=seed)
    for ep in range(episodes):
        r = env.reset_batched(want_obs=True, want_state=True)
        rc = c.reset(rng_step=b.rng_step - 1)
        assert np.array_equal(r["obs"].cpu().numpy(), rc["obs"])
        assert np.array_equal(r["state"].cpu().numpy()[:, : s.S], rc["state"])
        for t in range(steps):
            rs = b.rng_step
            a = b.sample_actions(p_act)
            ac = c.sample_actions(rs, p=p_act)
            if kind == "comb":
                assert np.array_equal(a.cpu().numpy(), pack(ac, s.C)), (ep, t)
            else:
                assert np.array_equal(a.cpu().numpy(), ac), (ep, t)
            rs = b.rng_step
            out = env.step_batched(a, want_obs=True, want_state=True, want_ack=True, want_success=True)
            oc = c.step(ac, rng_step=rs)
            assert np.array_equal(out["obs"].cpu().numpy(), oc["obs"]), (ep, t)
            assert np.array_equal(out["state"].cpu().numpy()[:, : s.S], oc["state"]), (ep, t)
            assert np.array_equal(out["reward"].cpu().numpy(), oc["reward"]), (ep, t)
            assert np.array_equal(out["ack"].cpu().numpy().astype(np.float64), oc["ack"]), (ep, t)
            assert np.array_equal(out["success"].cpu().numpy(), oc["success"]), (ep, t)
            assert np.array_equal(b.buffers_host(), c.buf), (ep, t)
            assert np.array_equal(b.channels_host(), c.chan), (ep, t)
            assert np.array_equal(b.received.cpu().numpy().astype(np.uint32), c.recv)
            assert np.array_equal(b.discarded.cpu().numpy().astype(np.uint32), c.disc)
            if kind == "chsel":
                assert np.array_equal(b.sel_quality.cpu().numpy().astype(np.uint32), c.selq)
                assert np.array_equal(b.sel_count.cpu().numpy().astype(np.uint32), c.seln)


@pytest.mark.parametrize("name", ["comb_6x8_setup8", "comb_8x8_ippo", "comb_64x8_tiled", "comb_12x4_xpnagents",
                                  "comb_4x3_periodic", "comb_1x1_heavy", "chsel_16x4", "chsel_5x16_het",
                                  "chsel_6x2_mixed"])
def test_philox_matches_c_oracle(name):
    z = np.load(os.path.join(GOLDEN, f"env_{name}.npz"))
    params = load_params(z)
    params["episode_length"] = 15
    _philox_case(str(z["kind"]), params, E=257, steps=15, seed=20261015)


@pytest.mark.parametrize("N,C,D", [(65, 8, 7), (128, 8, 14), (256, 8, 7), (100, 16, 20), (96, 32, 3),
                                   (512, 8, 7), (1024, 2, 4)])  # N > 64 stages an env's obs + state in LDS
def test_philox_large_agent_counts(N, C, D):
    """N > 64: one env per workgroup (up to 1,024 agents, 16 waves)."""
    params = dict(n_agents=N, n_channels=C, deadlines=np.array([D, max(1, D // 2)] * (N // 2) + [D] * (N % 2)),
                  lbdas=np.full(N, 0.3), episode_length=6, traffic_model="aperiodic",
                  channel_switch=np.full((N, C), 0.4))
    _philox_case("comb", params, E=33, steps=6, seed=7, p_act=0.05)
    params_c = dict(params, channel_switch=np.full(C + 1, 0.4))
    params_c.pop("homogeneous_size", None)
    if C <= 31:
        _philox_case("chsel", params_c, E=33, steps=6, seed=8)


# ------------------------------------------------- reference-API structures
@pytest.mark.parametrize("name", ["comb_6x8_setup8", "comb_8x8_ippo", "chsel_5x16_het"])
def test_reference_api_structures(name):
    from oracle.c_oracle import COracle
    z = np.load(os.path.join(GOLDEN, f"env_{name}.npz"))
    kind = str(z["kind"])
    params = load_params(z)
    params["episode_length"] = 20
    env = make_env(kind, params, seed=99)
    c = COracle(kind, params, n_envs=1, seed=99)
    s = env.spec
    rng = np.random.default_rng(0)
    for ep in range(2):
        obs, state = env.reset()
        rc = c.reset(rng_step=env.batch().rng_step - 1)
        assert isinstance(obs, list) and len(obs) == s.N
        for k in range(s.N):
            assert obs[k].dtype == np.float64 and obs[k].shape == (env.observation_space[k].shape[0],)
            assert np.array_equal(obs[k].astype(np.float32), rc["obs"][0, k, : s.obs_len[k]])
        assert np.array_equal(np.concatenate(state).astype(np.float32), rc["state"][0])
        assert np.concatenate(state).shape == env.state_space.shape
        done = False
        while not done:
            if kind == "comb":
                a = (rng.random((s.N, s.C)) < 0.3).astype(np.float32)
                ac = a[None].astype(np.uint8)
            else:
                a = rng.integers(0, s.C + 1, size=s.N)
                ac = a[None].astype(np.uint8)
            rs = env.batch().rng_step
            obs, state, rew, done, info = env.step(a)
            oc = c.step(ac, rng_step=rs)
            assert rew.dtype == np.int64 and rew.shape == (s.N,) and np.all(rew == oc["reward"][0])
            assert isinstance(done, bool) and info == {}
            for k in range(s.N):
                o32 = obs[k].astype(np.float32)
                assert np.array_equal(o32, oc["obs"][0, k, : s.obs_len[k]])
            if kind == "chsel":
                for k in range(s.N):  # float64 1/n feedback exactly like the reference
                    assert np.array_equal(obs[k][s.d[k]:], oc["ack"][0])
            assert np.array_equal(np.concatenate(state).astype(np.float32), oc["state"][0])
        assert np.array_equal(env.received_packets, c.recv[0].astype(np.float64))
        assert np.array_equal(env.discarded_packets, c.disc[0].astype(np.float64))
        recv, disc = c.recv[0].astype(np.float64), c.disc[0].astype(np.float64)
        u = np.where(recv > 0, 1 - disc / np.where(recv > 0, recv, 1), 1.0)
        assert env.compute_jains() == pytest.approx(u.sum() ** 2 / s.N / (u ** 2).sum(), abs=1e-15)
        assert env.compute_urllc() == pytest.approx(1 - disc.sum() / recv.sum(), abs=1e-15)


def test_reference_api_errors():
    from envs.combinatorial_env import CombinatorialEnv
    e = CombinatorialEnv(3, 2, np.array([3, 3, 3]), np.ones(3), traffic_model="bogus")
    with pytest.raises(ValueError, match="traffic model not supported"):
        e.reset()
    e = CombinatorialEnv(3, 2, np.array([3, 3, 3]), np.ones(3), traffic_model="heterogeneous", periodic_devices=[])
    with pytest.raises(AssertionError):
        e.reset()


# ------------------------------------------------------------- full size
def _config3_params(episode_length=200):
    from d2dhip.spec import EnvSpec  # noqa: F401
    import json
    cs8 = np.array(json.load(open(os.path.join(os.path.dirname(GOLDEN), "..", "d2d-ppo_amd", "combinatorial_load",
                                               "channel_switch_8.json")))["__nd__"])
    N = 64
    return dict(n_agents=N, n_channels=8, deadlines=np.array([7, 14] * (N // 2)), lbdas=np.full(N, 0.5),
                period=np.full(N, 2), arrival_probs=np.resize(np.array([.2, .4, .8, 1, 1, 1]), N), offsets=np.zeros(N),
                episode_length=episode_length, traffic_model="heterogeneous", homogeneous_size=True,
                periodic_devices=[k for k in range(N) if k % 6 < 3], channel_switch=np.resize(cs8, (N, 8)))


def test_full_size_bit_exact_slots():
    """64 agents x 8 channels x 65536 envs: HIP == C oracle, bit for bit, over 6 slots."""
    from oracle.c_oracle import COracle
    params = _config3_params()
    E = 65536
    env = make_env("comb", params, n_envs=E, device="cuda", seed=42)
    b = env.batch()
    c = COracle("comb", params, n_envs=E, seed=42, nthreads=16)
    r = env.reset_batched(want_obs=True, want_state=False)
    rc = c.reset(rng_step=0, want_state=False)
    assert np.array_equal(r["obs"].cpu().numpy(), rc["obs"])
    for t in range(6):
        rs = b.rng_step
        a = b.sample_actions(0.1)
        ac = c.sample_actions(rs, p=0.1)
        rs = b.rng_step
        out = env.step_batched(a, want_obs=True, want_state=(t == 5))
        oc = c.step(ac, rng_step=rs, want_state=(t == 5))
        assert np.array_equal(out["obs"].cpu().numpy(), oc["obs"]), t
        assert np.array_equal(out["reward"].cpu().numpy(), oc["reward"]), t
        if t == 5:
            assert np.array_equal(out["state"].cpu().numpy()[:, : b.spec.S], oc["state"])
    assert np.array_equal(b.buffers_host(), c.buf)
    assert np.array_equal(b.channels_host(), c.chan)


def test_full_size_record_slots_bit_exact():
    """The headline instantiation itself (the bench's `value`): 64 agents x 8 channels x 65,536 envs
    emitting the compact obs record (256-lane record-only blocks, comb_kernel<u8, 4, false, 8, false>
    in record mode).  Over 6 slots incl. the reset, the decoded record equals the C oracle's fp32 obs
    bit for bit, and rewards / buffers / channels match."""
    from oracle.c_oracle import COracle
    params = _config3_params()
    E = 65536
    env = make_env("comb", params, n_envs=E, device="cuda", seed=43)
    b = env.batch()
    c = COracle("comb", params, n_envs=E, seed=43, nthreads=16)
    rec = b.record
    b.reset(want_obs=True, out_obs=rec)
    rc = c.reset(rng_step=0, want_state=False)
    assert np.array_equal(rec.decode().cpu().numpy(), rc["obs"])
    rew = torch.empty((E,), dtype=torch.int32, device=b.device)
    for t in range(6):
        rs = b.rng_step
        a = b.sample_actions(0.1)
        ac = c.sample_actions(rs, p=0.1)
        rs = b.rng_step
        b.step(a, want_obs=True, out_obs=rec, out_reward=rew)
        oc = c.step(ac, rng_step=rs, want_state=False)
        assert np.array_equal(rec.decode().cpu().numpy(), oc["obs"]), t
        assert np.array_equal(rew.cpu().numpy(), oc["reward"]), t
    assert np.array_equal(b.buffers_host(), c.buf)
    assert np.array_equal(b.channels_host(), c.chan)


def test_full_size_episode_invariants():
    """Whole episode at 64 x 8 x 65536: packet conservation, reward bounds, ACK alphabet."""
    params = _config3_params()
    E = 65536
    env = make_env("comb", params, n_envs=E, device="cuda", seed=3)
    b = env.batch()
    env.reset_batched(want_obs=False)
    delivered = torch.zeros(E, dtype=torch.int64, device=b.device)
    done = False
    while not done:
        a = b.sample_actions(0.05)
        out = env.step_batched(a, want_obs=True, want_ack=True)
        rw = out["reward"]
        assert int(rw.min()) >= 0 and int(rw.max()) <= min(64, 8)
        ack = out["ack"]
        assert bool(((ack >= -1) & (ack <= 1)).all())
        # an ACK of 1 on channel c <=> exactly one success there; successes <= #channels with ACK 1
        assert bool(((ack == 1).sum(1) >= rw).all())
        delivered += rw.long()
        done = out["done"]
    recv = b.received.long().sum(1)
    disc = b.discarded.long().sum(1)
    buf = torch.from_numpy(b.buffers_host().astype(np.int64)).to(b.device).sum((1, 2))
    assert bool((recv == disc + delivered + buf).all())
    assert int(delivered.sum()) > 0 and int(disc.sum()) > 0


def test_oversized_env_rejected_loudly():
    """An env whose obs + state rows exceed the workgroup's LDS (N > 64 stages the whole env) is
    refused with NotImplementedError before any launch, not computed wrongly."""
    N, C, D = 1024, 32, 32
    env = make_env("comb", dict(n_agents=N, n_channels=C, deadlines=np.full(N, D), lbdas=np.full(N, 0.1),
                                episode_length=4, channel_switch=np.full((N, C), 0.4)), n_envs=2, device="cuda", seed=1)
    with pytest.raises(NotImplementedError, match="LDS"):
        env.reset_batched(want_obs=True, want_state=True)
