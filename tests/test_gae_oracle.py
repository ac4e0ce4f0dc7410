"""Pin the GAE/returns oracle to the reference's golden vectors (CPU)."""
# tolerance: 1e-5 absolute (BASELINE.json north_star: floats within 1e-5)
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle.gae_oracle import compute_gae_seq, discount_rewards_seq, gae_returns_batched


@pytest.fixture(scope="module")
def z():
    return np.load(os.path.join(GOLDEN, "gae_returns.npz"))


@pytest.mark.parametrize("case", ["small", "mid", "big"])
@pytest.mark.parametrize("gamma", [0.6, 0.99])
def test_gae_oracle_matches_reference(z, case, gamma):
    rew, val, done = z[f"{case}_rew"], z[f"{case}_val"], z[f"{case}_done"]
    adv = compute_gae_seq(rew, done, val, gamma, 0.97)
    ret = discount_rewards_seq(rew, gamma, done)
    np.testing.assert_allclose(adv, z[f"{case}_g{gamma}_adv"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(ret, z[f"{case}_g{gamma}_ret"], rtol=0, atol=1e-5)
    # D2D path: 1-D mean reward with float32 critic values (d2d_ppo.py:425-426, 333-339)
    adv1 = compute_gae_seq(rew.mean(1)[:, None], done, z[f"{case}_v32"][:, None], gamma, 0.97)[:, 0]
    np.testing.assert_allclose(adv1, z[f"{case}_g{gamma}_adv1d"], rtol=0, atol=1e-5)
    ret1 = discount_rewards_seq(rew, gamma, done).mean(1)
    np.testing.assert_allclose(ret1, z[f"{case}_g{gamma}_ret1d"], rtol=0, atol=1e-5)


@pytest.mark.parametrize("case,gamma", [("zerostd", 0.9), ("alldone", 0.8)])
def test_gae_oracle_edge_cases(z, case, gamma):
    rew, val, done = z[f"{case}_rew"], z[f"{case}_val"], z[f"{case}_done"]
    np.testing.assert_allclose(compute_gae_seq(rew, done, val, gamma, 0.97), z[f"{case}_adv"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(discount_rewards_seq(rew, gamma, done), z[f"{case}_ret"], rtol=0, atol=1e-5)


def test_batched_equals_concatenated_sequence(z):
    # [T][E][cols] env-major batch == the reference run on the concatenated episodes
    rew, val, done = z["mid_rew"], z["mid_val"], z["mid_done"]  # T=400 = 2 episodes of 200
    T2 = 200
    rb = np.stack([rew[:T2, 0], rew[T2:, 0]], axis=1)            # [T2][E=2]
    vb = np.stack([val[:T2], val[T2:]], axis=1)                  # [T2][2][cols]
    adv, ret = gae_returns_batched(rb, vb, done[:T2], 0.6, 0.97)
    np.testing.assert_allclose(np.concatenate([adv[:, 0], adv[:, 1]]), z["mid_g0.6_adv"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(np.concatenate([ret[:, 0], ret[:, 1]]), z["mid_g0.6_ret"], rtol=0, atol=1e-5)
