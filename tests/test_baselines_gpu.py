"""Baselines on the vectorised env (pytest -m gpu).

`run()` with n_envs > 1 runs E episodes per wave on the GPU (device policy + env kernel +
device metric reductions).  Each case is re-run on the CPU oracles with the same Philox
counters (numpy oracle for the D2DEnv, C oracle for comb / chsel) and the reference's
per-episode statistics; the returned tuples must agree (integer-derived terms exactly,
Jain's mean to 1e-12)."""
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


def _jains(recv, disc):
    u = np.where(recv > 0, 1 - disc / np.maximum(recv, 1), 1.0)
    return u.sum(1) ** 2 / recv.shape[1] / (u ** 2).sum(1)


def _oracle_run(o, policy, waves, L, N, samples, extra):
    """Walk the EnvBatch's rng_step sequence: reset(r), then per slot [sample(r)] step(r)."""
    rs = 0
    recv, disc, jains, ext, rew = [], [], [], [], []
    for _ in range(waves):
        o.reset(rng_step=rs)
        rs += 1
        acc = np.zeros(o.E, dtype=np.int64)
        for _t in range(L):
            a = policy(o, rs)
            if samples:
                rs += 1
            out = o.step(a, rng_step=rs)
            rs += 1
            acc += np.asarray(out["reward"] if "reward" in out else out["rewards"]).astype(np.int64)
        r = np.asarray(o.recv if hasattr(o, "recv") else o.received, dtype=np.float64)
        d = np.asarray(o.disc if hasattr(o, "disc") else o.discarded, dtype=np.float64)
        recv.append(r.sum(1)), disc.append(d.sum(1)), jains.append(_jains(r, d)), rew.append(acc * N)
        ext.append(extra(o))
    cat = np.concatenate
    return cat(recv), cat(disc), cat(jains), cat(ext), cat(rew)


def _check(res, ref, extra_kind):
    recv, disc, jains, ext, rew = ref
    assert res[0] == 1 - np.sum(disc) / np.sum(recv)
    assert abs(res[1] - np.mean(jains)) < 1e-12
    assert res[2] == (np.mean(ext) if extra_kind == "channel_score" else np.sum(ext))
    assert res[3] == np.mean(rew)


def _d2denv(E, L, seed):
    from envs.env import D2DEnv
    N = 6
    p = dict(n_agents=N, deadlines=np.array([3, 5, 4, 3, 6, 2]), lbdas=np.full(N, 0.25), episode_length=L,
             channel_switch=0.3, neighbourhoods=[[k, (k + 1) % N] for k in range(N)])
    return D2DEnv(**p, n_envs=E, device="cuda", seed=seed), p


def test_gf_access_on_d2denv_matches_oracle():
    from algorithms.baselines import GFAccess
    from oracle import philox
    from oracle.env_oracle import EnvOracle
    E, L, seed = 48, 20, 5
    env, p = _d2denv(E, L, seed)
    gf = GFAccess(env, transmission_prob=0.35)
    res = gf.run(2 * E - 10)                                    # 2 waves, ragged last wave
    o = EnvOracle("single", p, n_envs=E, seed=seed)
    envs = np.arange(E, dtype=np.uint64)

    def policy(o, rs):
        w = philox.words(envs[:, None], np.arange(6, dtype=np.uint64)[None, :], rs, philox.STREAM_ACTION, 1,
                         seed)[..., 0]
        return ((w < philox.threshold(0.35)) & (o.buffers.sum(2) > 0)).astype(np.int64)

    ref = _oracle_run(o, policy, 2, L, 6, True, lambda o: o.channel_errors.astype(np.float64))
    _check(res, tuple(x[: 2 * E - 10] for x in ref), "channel_errors")


def test_edf_on_d2denv_matches_oracle():
    from algorithms.baselines import EarliestDeadlineFirstScheduler
    from oracle.env_oracle import EnvOracle
    E, L, seed = 40, 25, 9
    env, p = _d2denv(E, L, seed)
    edf = EarliestDeadlineFirstScheduler(env)
    res = edf.run(E)
    o = EnvOracle("single", p, n_envs=E, seed=seed)
    ref_edf = EarliestDeadlineFirstScheduler(type("E", (), {"n_agents": 6})())

    def policy(o, rs):
        return np.stack([ref_edf.act(o.buffers[e]) for e in range(o.E)]).astype(np.int64)

    ref = _oracle_run(o, policy, 1, L, 6, False, lambda o: o.channel_errors.astype(np.float64))
    _check(res, ref, "channel_errors")
    assert res[2] > 0                                            # EDF ignores the channel: errors happen
    # use_channel hides agents on a bad channel: fewer channel errors
    env2, _ = _d2denv(E, L, seed)
    res2 = EarliestDeadlineFirstScheduler(env2, use_channel=True).run(E)
    assert res2[2] < res[2]


def test_combinatorial_random_access_matches_c_oracle():
    from algorithms.baselines import CombinatorialRandomAccess
    from envs.combinatorial_env import CombinatorialEnv
    from oracle.c_oracle import COracle
    N, C, E, L, seed = 8, 4, 64, 15, 3
    p = dict(n_agents=N, n_channels=C, deadlines=np.array([4, 7] * 4), lbdas=np.full(N, 0.3), episode_length=L,
             channel_switch=np.full((N, C), 0.3))
    env = CombinatorialEnv(**p, n_envs=E, device="cuda", seed=seed)
    cra = CombinatorialRandomAccess(env, transmission_prob=0.2)
    res = cra.run(E)
    o = COracle("comb", p, n_envs=E, seed=seed)
    ref = _oracle_run(o, lambda o, rs: o.sample_actions(rs, p=0.2), 1, L, N, True,
                      lambda o: np.ones(o.E))
    _check(res, ref, "channel_score")


def test_random_access_on_chsel_matches_c_oracle():
    from algorithms.baselines import RandomAccess
    from envs.channel_selection_env import ChannelSelectionEnv
    from oracle.c_oracle import COracle
    N, C, E, L, seed = 6, 3, 32, 15, 4
    p = dict(n_agents=N, n_channels=C, deadlines=np.full(N, 4), lbdas=np.full(N, 0.3), episode_length=L,
             channel_switch=np.full(C + 1, 0.3))
    env = ChannelSelectionEnv(**p, n_envs=E, device="cuda", seed=seed)
    res = RandomAccess(env).run(E)
    o = COracle("chsel", p, n_envs=E, seed=seed)

    def policy(o, rs):
        return o.sample_actions(rs) * (o.buf.sum(2) > 0)

    def score(o):
        q, n = o.selq.astype(np.float64), o.seln.astype(np.float64)
        return np.where(n != 0, q / np.maximum(n, 1), 1.0)

    ref = _oracle_run(o, policy, 1, L, N, True, score)
    _check(res, ref, "channel_score")


def test_host_loop_runs_on_d2denv():
    """n_envs = 1: the reference loop (fixed to read the env's buffers) on the D2DEnv."""
    from algorithms.baselines import EarliestDeadlineFirstScheduler, GFAccess
    env, _ = _d2denv(1, 10, 2)
    for bl in (EarliestDeadlineFirstScheduler(env, use_channel=True), GFAccess(env, use_channel=True)):
        score, jains, losses, rew = bl.run(2)
        assert 0 <= score <= 1 and 0 < jains <= 1 + 1e-12 and losses >= 0
