"""Pin the C oracle (CPU checker / CPU baseline) to the golden vectors and to
the numpy oracle, and pin Philox4x32-10 to the Random123 known-answer vectors."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, env_fixture_names, load_params
from oracle import philox
from oracle.c_oracle import COracle
from oracle.env_oracle import EnvOracle


def test_philox_known_answers():
    # Random123 kat_vectors, philox4x32 10 rounds
    kat = [((0, 0, 0, 0), 0, (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 4, 0xffffffffffffffff, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0x299f31d0 << 32) | 0xa4093822,
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, want in kat:
        got = tuple(int(x) for x in philox.philox4x32_10(*ctr, key))
        assert got == want


def test_poisson_inversion_moments():
    r = philox.words(np.arange(200000, dtype=np.uint64), 0, 0, 1, 1, 99)[..., 0]
    for lam in (1 / 14, 0.5, 2.5):
        x = philox.poisson_inversion(r, lam, np.exp(-lam))
        assert abs(x.mean() - lam) < 0.02 * max(lam, 0.3)
        assert abs(x.var() - lam) < 0.05 * max(lam, 0.3)


def test_poisson_cdf_table_equals_inversion():
    """The kernels' Poisson draw searches spec.poisson_cdf_table (d2d_env_desc.poisson_cdf); it must
    equal the oracle's sequential inversion for every word r.  Checked on Philox words, on every
    threshold t and t + 1 (both sides of each boundary), on 0 / 2^32 - 1, and for the chunked
    four-entry search the kernel runs (common.h poisson_lookup)."""
    from d2dhip.spec import POISSON, SCHEDULED, poisson_cdf_table
    lams = np.array([1 / 14, 1 / 3.5, 0.5, 2.5, 9.0, 33.0, 64.0, 0.25])
    kinds = np.array([POISSON] * 7 + [SCHEDULED])
    t = poisson_cdf_table(lams, kinds)
    assert t.shape == (8, 256) and t.dtype == np.uint32
    assert (t[7] == 0xFFFFFFFF).all() and (t[:, 255] == 0xFFFFFFFF).all()
    assert (np.diff(t.astype(np.int64), axis=1) >= 0).all()
    rnd = philox.words(np.arange(50000, dtype=np.uint64), 3, 0, 1, 1, 7)[..., 0]
    for k in range(7):
        tk = t[k].astype(np.uint64)
        edge = np.concatenate([tk[:255], np.minimum(tk[:255] + 1, 0xFFFFFFFF)])
        r = np.concatenate([rnd, edge, np.array([0, 0xFFFFFFFF], dtype=np.uint64)])
        want = philox.poisson_inversion(r, lams[k], np.exp(-lams)[k])
        got = np.searchsorted(tk, r, side="left")                   # count of entries t[x] < r
        assert (got == want).all(), k
        x = np.zeros(r.shape, dtype=np.int64)                       # the kernel's chunked search
        live = np.ones(r.shape, dtype=bool)
        while live.any():
            q = np.stack([tk[np.minimum(x + i, 255)] for i in range(4)], axis=1)
            n = (r[:, None] > q).sum(axis=1)
            x = np.where(live, x + n, x)
            live &= n == 4
        assert (x == want).all(), k


def test_poisson_cdf_table_refuses_underflowing_means():
    """exp(-lam) underflows to 0 near lam = 745, where ceil(F_x * 2^32) - 1 would wrap: such means
    (and every mean past the uint8 cells' 64) are refused at table build time, not mis-tabulated."""
    from d2dhip.spec import POISSON, poisson_cdf_table
    for lam in (64.5, 800.0, np.inf, np.nan):
        with pytest.raises(NotImplementedError):
            poisson_cdf_table(np.array([0.5, lam]), np.array([POISSON, POISSON]))


@pytest.mark.parametrize("name", env_fixture_names())
def test_c_oracle_replays_reference(name):
    z = np.load(os.path.join(GOLDEN, f"env_{name}.npz"))
    kind = str(z["kind"])
    params = load_params(z)
    o = COracle(kind, params, n_envs=1)
    L = int(params["episode_length"])
    step = 0
    for ep in range(int(z["episodes"])):
        r = o.reset(arrivals=z["reset_arrivals"][ep][None])
        assert np.array_equal(r["obs"][0], z["reset_obs"][ep].astype(np.float32))
        assert np.array_equal(r["state"][0], z["reset_state"][ep].astype(np.float32))
        for t in range(L):
            out = o.step(z["actions"][step][None], rng_step=step + 1, flips=z["flips"][step][None],
                         arrivals=z["arrivals"][step][None])
            assert np.array_equal(o.buf[0], z["buffers"][step]), (ep, t)
            assert np.array_equal(o.chan[0], z["chan"][step]), (ep, t)
            assert np.array_equal(out["obs"][0], z["obs"][step].astype(np.float32)), (ep, t)
            assert np.array_equal(out["state"][0], z["state"][step].astype(np.float32)), (ep, t)
            assert np.array_equal(out["ack"][0], z["ack"][step].astype(np.float64)), (ep, t)
            assert out["reward"][0] == z["rewards"][step][0]
            assert np.array_equal(out["success"][0].astype(bool), z["success"][step])
            assert np.array_equal(o.recv[0], z["received"][step]) and np.array_equal(o.disc[0], z["discarded"][step])
            if kind == "chsel":
                assert o.selq[0] == z["sel_q"][step] and o.seln[0] == z["sel_n"][step]
            step += 1


@pytest.mark.parametrize("name", ["comb_6x8_setup8", "comb_4x3_periodic", "comb_16x8_aperiodic", "chsel_16x4",
                                  "chsel_5x16_het", "comb_1x1_heavy"])
def test_c_oracle_philox_matches_numpy_oracle(name):
    z = np.load(os.path.join(GOLDEN, f"env_{name}.npz"))
    kind = str(z["kind"])
    params = load_params(z)
    params["episode_length"] = 12
    E, seed, base = 5, 1234567, 77
    c = COracle(kind, params, n_envs=E, seed=seed, env_base=base)
    n = EnvOracle(kind, params, n_envs=E, seed=seed, env_base=base)
    rs = 0
    for ep in range(2):
        rc = c.reset(rng_step=rs)
        rn = n.reset(rng_step=rs)
        rs += 1
        assert np.array_equal(rc["obs"], rn["obs"].astype(np.float32))
        for t in range(12):
            act = c.sample_actions(rs, p=0.3)
            oc = c.step(act, rng_step=rs)
            on = n.step(act, rng_step=rs)
            rs += 1
            assert np.array_equal(c.buf, n.buffers), (ep, t)
            assert np.array_equal(c.chan, n.chan), (ep, t)
            assert np.array_equal(oc["obs"], on["obs"].astype(np.float32)), (ep, t)
            assert np.array_equal(oc["state"], on["state"].astype(np.float32)), (ep, t)
            assert np.array_equal(oc["reward"], on["rewards"])
            assert np.array_equal(c.recv, n.received) and np.array_equal(c.disc, n.discarded)


def test_sample_actions_rate():
    z = np.load(os.path.join(GOLDEN, "env_comb_64x8_tiled.npz"))
    c = COracle("comb", load_params(z), n_envs=512, seed=5)
    a = c.sample_actions(3, p=0.1)
    assert a.shape == (512, 64, 8) and abs(a.mean() - 0.1) < 0.005
