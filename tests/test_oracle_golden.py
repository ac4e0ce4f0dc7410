"""Pin the CPU oracle (oracle/env_oracle.py) to the reference's own outputs.

Every golden fixture was produced by running the reference envs in the build
container (tools/gen_fixtures.py); here the oracle replays the recorded random
draws and must reproduce every output exactly (integers bit-exact, obs/state
exact after the fp32 cast, chsel 1/n feedback exact in float64).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, env_fixture_names, load_params
from oracle.env_oracle import EnvOracle


@pytest.mark.parametrize("name", env_fixture_names())
def test_oracle_replays_reference(name):
    z = np.load(os.path.join(GOLDEN, f"env_{name}.npz"))
    kind = str(z["kind"])
    params = load_params(z)
    o = EnvOracle(kind, params, n_envs=1)
    s = o.spec
    assert s.S == int(z["state_dim"])
    assert np.array_equal(s.w + (2 * s.C if kind == "comb" else s.C + 1), z["obs_dims"])
    L = int(params["episode_length"])
    step = 0
    for ep in range(int(z["episodes"])):
        r = o.reset(arrivals=z["reset_arrivals"][ep][None].astype(np.int64))
        assert np.array_equal(r["buffers"][0], z["reset_buffers"][ep])
        assert np.array_equal(r["obs"][0], z["reset_obs"][ep])
        assert np.array_equal(r["state"][0], z["reset_state"][ep])
        assert np.array_equal(r["received"][0], z["reset_received"][ep])
        for t in range(L):
            out = o.step(z["actions"][step][None], flips=z["flips"][step][None].astype(np.int64),
                         arrivals=z["arrivals"][step][None].astype(np.int64))
            assert np.array_equal(out["buffers"][0], z["buffers"][step]), (ep, t)
            assert np.array_equal(out["chan"][0], z["chan"][step]), (ep, t)
            assert np.array_equal(out["ack"][0], z["ack"][step]), (ep, t)
            assert np.array_equal(np.full(s.N, out["rewards"][0]), z["rewards"][step]), (ep, t)
            assert np.array_equal(out["success"][0], z["success"][step]), (ep, t)
            assert np.array_equal(out["received"][0], z["received"][step]), (ep, t)
            assert np.array_equal(out["discarded"][0], z["discarded"][step]), (ep, t)
            assert bool(out["done"]) == bool(z["done"][step])
            if kind == "comb":
                assert np.array_equal(out["obs"][0].astype(np.float32), z["obs"][step]), (ep, t)
                assert np.array_equal(out["state"][0].astype(np.float32), z["state"][step]), (ep, t)
            else:
                assert np.array_equal(out["obs"][0], z["obs"][step]), (ep, t)
                assert np.array_equal(out["state"][0], z["state"][step]), (ep, t)
                assert out["sel_q"][0] == z["sel_q"][step] and out["sel_n"][0] == z["sel_n"][step]
            step += 1
        assert np.isclose(o.compute_jains()[0], z["metric_jains"][ep], rtol=0, atol=1e-15)
        assert np.isclose(o.compute_urllc()[0], z["metric_urllc"][ep], rtol=0, atol=1e-15)
        assert np.isclose(o.compute_channel_score()[0], z["metric_channel_score"][ep], rtol=0, atol=1e-15)
    assert step == z["actions"].shape[0]


def test_fixture_set_covers_survey_cases():
    names = env_fixture_names()
    for must in ("comb_6x8_setup8", "comb_8x8_ippo", "comb_64x8_tiled", "chsel_16x4", "chsel_5x16_het"):
        assert must in names


def d2denv_fixture_names():
    import glob
    return sorted(os.path.basename(p)[7:-4] for p in glob.glob(os.path.join(GOLDEN, "d2denv_*.npz")))


@pytest.mark.parametrize("name", d2denv_fixture_names())
def test_oracle_replays_reference_d2denv(name):
    """D2DEnv (envs/env.py): the oracle replays the recorded flips / arrivals and reproduces every
    output of the reference exactly (obs / state exact after the fp32 cast)."""
    z = np.load(os.path.join(GOLDEN, f"d2denv_{name}.npz"))
    params = load_params(z)
    o = EnvOracle("single", params, n_envs=1)
    s = o.spec
    assert s.S == int(z["state_dim"])
    assert np.array_equal(s.obs_len, z["obs_dims"])
    L = int(params["episode_length"])
    step = 0
    for ep in range(int(z["episodes"])):
        r = o.reset(arrivals=z["reset_arrivals"][ep][None].astype(np.int64))
        assert np.array_equal(r["buffers"][0], z["reset_buffers"][ep])
        assert np.array_equal(r["obs"][0].astype(np.float32), z["reset_obs"][ep])
        assert np.array_equal(r["state"][0].astype(np.float32), z["reset_state"][ep])
        for t in range(L):
            out = o.step(z["actions"][step][None], flips=z["flips"][step][None].astype(np.int64),
                         arrivals=z["arrivals"][step][None].astype(np.int64))
            assert np.array_equal(out["buffers"][0], z["buffers"][step]), (ep, t)
            assert np.array_equal(out["chan"][0], z["chan"][step]), (ep, t)
            assert out["ack"][0, 0] == z["ack"][step], (ep, t)
            assert np.array_equal(np.full(s.N, out["rewards"][0]), z["rewards"][step]), (ep, t)
            assert np.array_equal(out["success"][0], z["success"][step]), (ep, t)
            assert np.array_equal(out["received"][0], z["received"][step]), (ep, t)
            assert np.array_equal(out["discarded"][0], z["discarded"][step]), (ep, t)
            assert out["channel_errors"][0] == z["channel_errors"][step]
            assert out["n_collisions"][0] == z["n_collisions"][step]
            assert np.array_equal(out["obs"][0].astype(np.float32), z["obs"][step]), (ep, t)
            assert np.array_equal(out["state"][0].astype(np.float32), z["state"][step]), (ep, t)
            assert bool(out["done"]) == bool(z["done"][step])
            step += 1
        assert np.isclose(o.compute_jains()[0], z["metric_jains"][ep], rtol=0, atol=1e-15)
        assert np.isclose(o.compute_urllc()[0], z["metric_urllc"][ep], rtol=0, atol=1e-15)
        assert o.successful_transmissions[0] == z["metric_successful_transmissions"][ep]
    assert step == z["actions"].shape[0]
