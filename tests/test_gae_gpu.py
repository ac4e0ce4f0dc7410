"""GPU parity of the GAE / returns kernels (pytest -m gpu).

Tolerance: 1e-5 absolute on the normalised float32 outputs (BASELINE.json
north_star: floats within 1e-5), against the reference's golden vectors and,
at batch sizes, against the numpy oracle (oracle/gae_oracle.py) which is
itself pinned to the golden vectors.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
ATOL = 1e-5


@pytest.fixture(scope="module")
def z():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm GPU")
    return np.load(os.path.join(GOLDEN, "gae_returns.npz"))


def run(rew, val, done, gamma, **kw):
    from d2dhip.gae import gae_returns
    dev = "cuda"
    r = torch.from_numpy(np.ascontiguousarray(rew, dtype=np.float32)).to(dev)
    v = torch.from_numpy(np.ascontiguousarray(val, dtype=np.float32)).to(dev)
    d = torch.from_numpy(np.asarray(done, dtype=np.uint8)).to(dev)
    adv, ret = gae_returns(r, v, d, gamma, 0.97, **kw)
    return adv.cpu().numpy(), ret.cpu().numpy()


@pytest.mark.parametrize("case", ["small", "mid", "big"])
@pytest.mark.parametrize("gamma", [0.6, 0.99])
def test_gae_kernel_matches_reference(z, case, gamma):
    rew, val, done = z[f"{case}_rew"], z[f"{case}_val"], z[f"{case}_done"]
    T, N = val.shape
    # iPPO layout: one env, N agent columns, reward broadcast (the envs give every agent the same reward)
    adv, ret = run(rew[:, :1], val[:, None, :], done, gamma)
    np.testing.assert_allclose(adv[:, 0], z[f"{case}_g{gamma}_adv"], rtol=0, atol=ATOL)
    np.testing.assert_allclose(ret[:, 0], z[f"{case}_g{gamma}_ret"], rtol=0, atol=ATOL)
    # D2D layout: central critic, one column (d2d_ppo.py:425-426, 333-339)
    adv1, ret1 = run(rew[:, :1], z[f"{case}_v32"][:, None, None], done, gamma)
    np.testing.assert_allclose(adv1[:, 0, 0], z[f"{case}_g{gamma}_adv1d"], rtol=0, atol=ATOL)
    np.testing.assert_allclose(ret1[:, 0, 0], z[f"{case}_g{gamma}_ret1d"], rtol=0, atol=ATOL)


@pytest.mark.parametrize("case,gamma", [("zerostd", 0.9), ("alldone", 0.8)])
def test_gae_kernel_edge_cases(z, case, gamma):
    rew, val, done = z[f"{case}_rew"], z[f"{case}_val"], z[f"{case}_done"]
    adv, ret = run(rew[:, None, :], val[:, None, :], done, gamma)
    np.testing.assert_allclose(adv[:, 0], z[f"{case}_adv"], rtol=0, atol=ATOL)
    np.testing.assert_allclose(ret[:, 0], z[f"{case}_ret"], rtol=0, atol=ATOL)


@pytest.mark.parametrize("T,E,cols", [(200, 64, 8), (400, 256, 64), (200, 4096, 1)])
def test_gae_kernel_batched_vs_oracle(T, E, cols):
    from oracle.gae_oracle import gae_returns_batched
    rng = np.random.default_rng(T + E + cols)
    rew = rng.integers(0, 5, size=(T, E)).astype(np.float32)
    val = rng.normal(size=(T, E, cols)).astype(np.float32)
    done = np.zeros(T, dtype=bool)
    done[99::100] = True
    done[-1] = True
    adv, ret = run(rew, val, done, 0.6)
    adv_o, ret_o = gae_returns_batched(rew, val, done, 0.6, 0.97)
    np.testing.assert_allclose(adv, adv_o, rtol=0, atol=ATOL)
    np.testing.assert_allclose(ret, ret_o, rtol=0, atol=ATOL)


def test_gae_kernel_size_independent_properties():
    """Full config-3 rollout size (T=200, E=65536, 64 columns): normalised columns have
    mean 0 / std 1 (ddof 0 for adv, 1 for ret) and the raw scan obeys its recursion."""
    from d2dhip.gae import gae_returns
    T, E, cols = 200, 65536, 64
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    rew = torch.randint(0, 4, (T, E), device="cuda", generator=g).float()
    val = torch.randn((T, E, cols), device="cuda", generator=g)
    done = torch.zeros(T, dtype=torch.uint8, device="cuda")
    done[-1] = 1
    adv, ret = gae_returns(rew, val, done, 0.6, 0.97)
    a = adv.view(-1, cols).double()
    r = ret.view(-1, cols).double()
    assert float(a.mean(0).abs().max()) < 1e-5 and float((a.std(0, unbiased=False) - 1).abs().max()) < 1e-5
    assert float(r.mean(0).abs().max()) < 1e-5 and float((r.std(0, unbiased=True) - 1).abs().max()) < 1e-5
    adv_raw, ret_raw = gae_returns(rew, val, done, 0.6, 0.97, normalize_adv=False, normalize_ret=False)
    # R_t = r_t + gamma R_{t+1} inside an episode; every column sees the same reward
    lhs = ret_raw[:-1].double()
    rhs = rew[:-1, :, None].double() + 0.6 * ret_raw[1:].double()
    assert float((lhs - rhs).abs().max()) < 1e-4


@pytest.mark.parametrize("T,E,cols,rcols", [(200, 64, 8, 1), (400, 33, 64, 1), (50, 300, 5, 5), (120, 1, 4, 1)])
def test_gae_kernel_tce_layout(T, E, cols, rcols):
    """The [T][cols][E] entry points (values as the policy kernel writes them) give the [T][E][cols]
    results transposed, and match the oracle (ragged E, per-column and broadcast rewards)."""
    from oracle.gae_oracle import gae_returns_batched
    rng = np.random.default_rng(T * 7 + E + cols)
    rew = rng.integers(0, 5, size=(T, E) if rcols == 1 else (T, E, cols)).astype(np.float32)
    val = rng.normal(size=(T, E, cols)).astype(np.float32)
    done = np.zeros(T, dtype=bool)
    done[T // 2 - 1] = True
    done[-1] = True
    adv, ret = run(rew, val, done, 0.6)
    rew_tce = rew if rcols == 1 else np.ascontiguousarray(rew.transpose(0, 2, 1))
    adv_t, ret_t = run(rew_tce, np.ascontiguousarray(val.transpose(0, 2, 1)), done, 0.6, layout="tce")
    np.testing.assert_allclose(adv_t.transpose(0, 2, 1), adv, rtol=0, atol=1e-6)
    np.testing.assert_allclose(ret_t.transpose(0, 2, 1), ret, rtol=0, atol=1e-6)
    if rcols == 1:
        adv_o, ret_o = gae_returns_batched(rew, val, done, 0.6, 0.97)
        np.testing.assert_allclose(adv_t.transpose(0, 2, 1), adv_o, rtol=0, atol=ATOL)
        np.testing.assert_allclose(ret_t.transpose(0, 2, 1), ret_o, rtol=0, atol=ATOL)
