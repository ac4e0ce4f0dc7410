"""d2d_critic_dpre_split (ABI v7): the D2D central critic's backward glue (algorithms/d2d_ppo.py
_critic_split_backward; the reference's value_loss.backward() through its central Value net,
/root/reference/algorithms/d2d_ppo.py:95-98, 208-216) against the torch ops it replaced."""
import pytest
import torch

from d2dhip import _lib

pytestmark = pytest.mark.gpu


def torch_ref(pre, w2, dv):
    dpre = torch.where(pre > 0, w2[:, None] * dv[None, :], torch.zeros_like(pre))
    dh = dpre.to(torch.bfloat16)
    dm = (dpre - dh.float()).to(torch.bfloat16)
    return torch.cat([dh, dm], 0), dpre.double().sum(1), (torch.relu(pre).double() * dv.double()[None, :]).sum(1)


@pytest.mark.parametrize("H,B", [(64, 819_200), (64, 1), (16, 5), (128, 12_345), (7, 4_096 * 3 + 1)])
def test_dpre_split_matches_torch(H, B):
    g = torch.Generator(device="cuda").manual_seed(H * 7 + B)
    pre = torch.randn((H, B), device="cuda", generator=g)
    pre[:, ::7] = 0.0  # relu'(0) = 0, as torch.where(pre > 0, ...)
    w2 = torch.randn(H, device="cuda", generator=g) * 0.1
    dv = torch.randn(B, device="cuda", generator=g) * 1e-3
    lib = _lib.require_gpu()
    G = int(lib.d2d_critic_dpre_blocks(B))
    dhm = torch.empty((2 * H, B), dtype=torch.bfloat16, device="cuda")
    part = torch.empty((G, 2 * H), dtype=torch.float32, device="cuda")
    _lib.check(lib.d2d_critic_dpre_split(H, B, pre.data_ptr(), w2.data_ptr(), dv.data_ptr(), dhm.data_ptr(),
                                         part.data_ptr(), G, _lib.stream_ptr()), "d2d_critic_dpre_split")
    ref_dhm, ref_db1, ref_gw2 = torch_ref(pre, w2, dv)
    assert torch.equal(dhm, ref_dhm)  # the split parts bit for bit
    sums = part.sum(0).double()
    # fp32 block sums vs float64: relative to the sum of magnitudes
    mag_db1 = (torch.where(pre > 0, w2[:, None] * dv[None, :], torch.zeros_like(pre))).abs().double().sum(1)
    mag_gw2 = (torch.relu(pre) * dv[None, :]).abs().double().sum(1)
    assert bool(((sums[:H] - ref_db1).abs() <= 1e-5 * mag_db1 + 1e-12).all())
    assert bool(((sums[H:] - ref_gw2).abs() <= 1e-5 * mag_gw2 + 1e-12).all())


def test_dpre_split_rejects_wrong_block_count():
    lib = _lib.require_gpu()
    pre = torch.zeros((4, 100), device="cuda")
    rc = lib.d2d_critic_dpre_split(4, 100, pre.data_ptr(), pre.data_ptr(), pre.data_ptr(), pre.data_ptr(),
                                   pre.data_ptr(), int(lib.d2d_critic_dpre_blocks(100)) + 1, _lib.stream_ptr())
    assert rc != 0
