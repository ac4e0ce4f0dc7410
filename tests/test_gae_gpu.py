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


@pytest.mark.parametrize("layout,T,E,cols,rcols", [("tce", 200, 1000, 64, 1), ("tec", 200, 333, 64, 1),
                                                   ("tec", 50, 300, 5, 5), ("tec", 120, 1, 4, 1),
                                                   ("tec", 30, 7, 300, 1), ("tce", 17, 4097, 3, 3)])
def test_gae_scan_moments_fused_stats(layout, T, E, cols, rcols):
    """d2d_gae_scan_moments (the scan with both outputs' column moments fused in): adv / ret bitwise
    equal to the plain scan, (n, sum, M2) per column equal to float64 statistics of the stored fp32
    outputs (1e-12 relative), and bitwise reproducible run to run (fixed-order combines)."""
    from d2dhip import _lib
    lib = _lib.require_gpu()
    dev = "cuda"
    g = torch.Generator(device=dev)
    g.manual_seed(T + E + cols)
    tce = layout == "tce"
    vshape = (T, cols, E) if tce else (T, E, cols)
    val = torch.randn(vshape, device=dev, generator=g) * 3 + 1
    rew = torch.randint(0, 5, (T, E) if rcols == 1 else vshape, device=dev, generator=g).float()
    done = torch.zeros(T, dtype=torch.uint8, device=dev)
    done[T // 2] = 1
    done[-1] = 1
    lay = 1 if tce else 0

    def fused():
        adv, ret = torch.empty_like(val), torch.empty_like(val)
        mom = torch.empty((2, 3, cols), dtype=torch.float64, device=dev)
        ws = torch.empty(int(lib.d2d_gae_moments_workspace(E, cols, lay)), dtype=torch.float64, device=dev)
        _lib.check(lib.d2d_gae_scan_moments(T, E, cols, rcols, rew.data_ptr(), val.data_ptr(), done.data_ptr(), 0.6,
                                            0.97, 1, lay, adv.data_ptr(), ret.data_ptr(), mom.data_ptr(),
                                            ws.data_ptr(), ws.numel(), _lib.stream_ptr()), "scan_moments")
        return adv, ret, mom

    a1, r1, m1 = fused()
    a2, r2, m2 = fused()
    assert torch.equal(a1, a2) and torch.equal(r1, r2) and torch.equal(m1, m2)
    a0, r0 = torch.empty_like(val), torch.empty_like(val)
    scan = lib.d2d_gae_scan_tce if tce else lib.d2d_gae_scan
    _lib.check(scan(T, E, cols, rcols, rew.data_ptr(), val.data_ptr(), done.data_ptr(), 0.6, 0.97, 1, a0.data_ptr(),
                    r0.data_ptr(), _lib.stream_ptr()), "scan")
    assert torch.equal(a1, a0) and torch.equal(r1, r0)
    for k, x in enumerate((a1, r1)):
        xc = (x.permute(1, 0, 2) if tce else x.permute(2, 0, 1)).reshape(cols, -1).double()   # [cols][T*E]
        assert torch.equal(m1[k, 0], torch.full((cols,), float(T * E), dtype=torch.float64, device=dev))
        torch.testing.assert_close(m1[k, 1], xc.sum(1), rtol=1e-12, atol=1e-9)
        torch.testing.assert_close(m1[k, 2], ((xc - xc.mean(1, keepdim=True)) ** 2).sum(1), rtol=1e-11, atol=1e-9)


def test_gae_constant_column_keeps_gate_closed():
    """Quirk Q2 on the fused statistics: one constant column (std exactly 0) disables the
    normalisation of every column, for adv (ddof 0) and ret (ddof 1) alike."""
    from d2dhip.gae import gae_returns
    T, E, cols = 40, 300, 3
    dev = "cuda"
    val = torch.randn(T, E, cols, device=dev)
    val[..., 1] = 0.0
    rew = torch.zeros(T, E, cols, device=dev)
    rew[..., 0] = 1.0
    done = torch.zeros(T, dtype=torch.uint8, device=dev)
    done[-1] = 1
    adv_raw, ret_raw = gae_returns(rew, val, done, 0.5, 0.97, normalize_adv=False, normalize_ret=False, last_shard=False)
    adv, ret = gae_returns(rew, val, done, 0.5, 0.97, last_shard=False)
    # column 1: rewards 0, values 0 -> adv = ret = 0 everywhere (std 0) -> no column is normalised
    assert torch.equal(adv, adv_raw) and torch.equal(ret, ret_raw)


@pytest.mark.parametrize("layout,T,E,cols,rcols", [("tce", 200, 1000, 64, 1), ("tec", 200, 333, 64, 1),
                                                   ("tec", 50, 300, 5, 5), ("tce", 17, 4097, 3, 3),
                                                   ("tec", 120, 1, 4, 1)])
@pytest.mark.parametrize("which", ["both", "adv", "ret"])
def test_gae_two_scan_normalised_equals_scan_plus_normalise(layout, T, E, cols, rcols, which):
    """ABI 9: the moments-only scan + d2d_gae_scan_normalized (gae_returns' path) write bitwise the
    outputs of the fused scan + d2d_normalize_pair (the ABI 8 path), for both outputs normalised or
    only one (the other written raw), and the moments-only scan's statistics equal the fused scan's."""
    from d2dhip import _lib
    from d2dhip.gae import gae_returns, moments_stats
    lib = _lib.require_gpu()
    dev = "cuda"
    g = torch.Generator(device=dev)
    g.manual_seed(T * 3 + E + cols)
    tce = layout == "tce"
    vshape = (T, cols, E) if tce else (T, E, cols)
    val = torch.randn(vshape, device=dev, generator=g) * 2 - 0.5
    rew = torch.randint(0, 5, (T, E) if rcols == 1 else vshape, device=dev, generator=g).float()
    done = torch.zeros(T, dtype=torch.uint8, device=dev)
    done[T // 3] = 1
    done[-1] = 1
    lay = 1 if tce else 0
    na, nr = which in ("both", "adv"), which in ("both", "ret")
    # ABI 8 path
    adv0, ret0 = torch.empty_like(val), torch.empty_like(val)
    mom = torch.empty((2, 3, cols), dtype=torch.float64, device=dev)
    ws = torch.empty(int(lib.d2d_gae_moments_workspace(E, cols, lay)), dtype=torch.float64, device=dev)
    _lib.check(lib.d2d_gae_scan_moments(T, E, cols, rcols, rew.data_ptr(), val.data_ptr(), done.data_ptr(), 0.6, 0.97,
                                        1, lay, adv0.data_ptr(), ret0.data_ptr(), mom.data_ptr(), ws.data_ptr(),
                                        ws.numel(), _lib.stream_ptr()), "scan_moments")
    mom_only = torch.empty_like(mom)
    _lib.check(lib.d2d_gae_scan_moments(T, E, cols, rcols, rew.data_ptr(), val.data_ptr(), done.data_ptr(), 0.6, 0.97,
                                        1, lay, None, None, mom_only.data_ptr(), ws.data_ptr(), ws.numel(),
                                        _lib.stream_ptr()), "scan_moments (moments only)")
    assert torch.equal(mom, mom_only)
    args, keep = [], []
    for x, do, k, ddof in ((adv0, na, 0, 0), (ret0, nr, 1, 1)):
        if do:
            st = moments_stats(mom[k], ddof, T * E)
            keep.append(st)
            args += [x.data_ptr()] + [t.data_ptr() for t in st]
        else:
            args += [None] * 4
    _lib.check(lib.d2d_normalize_pair(T, E, cols, lay, *args, _lib.stream_ptr()), "normalize_pair")
    # ABI 9 path
    adv1, ret1 = gae_returns(rew, val, done, 0.6, 0.97, normalize_adv=na, normalize_ret=nr, layout=layout)
    torch.cuda.synchronize()
    assert torch.equal(adv1, adv0) and torch.equal(ret1, ret0)
