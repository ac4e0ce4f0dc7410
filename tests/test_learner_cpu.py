"""CPU unit tests of the learners' host-side math (no HIP calls): the
agent-stacked networks, the GRU cell, the HAPPO prefix product and the RNN
window builder.  Tolerance 1e-5 absolute (1e-6 where noted) against plain
per-agent torch modules / the reference's golden windows."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from algorithms._core import Policy, RNN, StackedNets, Value, gru_window, rnn_windows
from algorithms.d2d_ppo import happo_chain


def _mods(cls, dims, *a, **kw):
    torch.manual_seed(0)
    return [cls(d, *a, **kw) for d in dims]


@pytest.mark.parametrize("kind", ["mlp", "rnn"])
def test_stacked_forward_equals_per_agent_modules(kind):
    dims = [23, 30, 23, 30, 19]
    if kind == "mlp":
        mods = _mods(Policy, dims, 8, 16)
        ref_out = None
    else:
        mods = _mods(RNN, dims, 8, 16, combinatorial=True)
    with torch.no_grad():
        ref = []
        x = torch.randn(len(dims), 7, 4, 30) if kind == "rnn" else torch.randn(len(dims), 7, 30)
        for k, (m, d) in enumerate(zip(mods, dims)):
            xk = x[k, ..., :d]
            ref.append(m(xk) if kind == "mlp" else m(xk))
        ref_out = torch.stack(ref)
    st = StackedNets(mods, dims, kind, "cpu", act="softmax" if kind == "mlp" else "sigmoid")
    xz = x.clone()
    for k, d in enumerate(dims):
        xz[k, ..., d:] = 0  # the env writes zeros past each agent's obs length
    with torch.no_grad():
        out = st.forward(xz)
        # modules now view the stacked storage and still agree
        again = torch.stack([m(xz[k, ..., :d]) for k, (m, d) in enumerate(zip(mods, dims))])
    torch.testing.assert_close(out, ref_out, rtol=0, atol=1e-6)
    torch.testing.assert_close(again, ref_out, rtol=0, atol=1e-6)


def test_gru_window_matches_torch_gru():
    torch.manual_seed(1)
    gru = torch.nn.GRU(11, 16, 1)
    x = torch.randn(5, 6, 11)  # batch, seq, in
    with torch.no_grad():
        out, _ = gru(x.permute(1, 0, 2))
        h = gru_window(x.unsqueeze(0), gru.weight_ih_l0[None], gru.weight_hh_l0[None], gru.bias_ih_l0[None],
                       gru.bias_hh_l0[None])[0]
    torch.testing.assert_close(h, out[-1], rtol=0, atol=1e-6)


def test_happo_prefix_equals_sequential_chain():
    torch.manual_seed(2)
    N, B = 6, 50
    adv = torch.randn(B)
    ratio = torch.exp(0.1 * torch.randn(N, B))
    perm = np.random.default_rng(0).permutation(N)
    M = happo_chain(adv, ratio, perm)
    cur = adv.clone()
    for j, i in enumerate(perm):          # d2d_ppo.py:429-436: M = ratio_i * M after agent i
        assert torch.equal(M[i], cur)
        cur = ratio[i] * cur


@pytest.mark.parametrize("variant", ["ippo_rnn_comb", "d2d_rnn_cat"])
def test_rnn_windows_match_reference(variant):
    z = np.load(os.path.join(GOLDEN, f"learner_{variant}.npz"))
    obs0 = torch.from_numpy(z["ro/obs0"])
    win = rnn_windows(obs0.unsqueeze(0), int(z["history_len"]), int(z["episode_length"]))[0]
    assert np.array_equal(win.numpy(), z["rnnwin/agent0"])


def test_stacked_grad_clip_equals_per_agent_clip():
    dims = [10, 10, 10]
    mods = _mods(Policy, dims, 4, 8)
    ref = _mods(Policy, dims, 4, 8)
    st = StackedNets(mods, dims, "mlp", "cpu", act="softmax")
    x = torch.randn(3, 20, 10) * 50
    loss = st.forward(x).pow(2).sum() * 100
    loss.backward()
    norms = st.grad_norm_clip_(20)
    for k, m in enumerate(ref):
        y = m(x[k]).pow(2).sum() * 100
        y.backward()
        tn = torch.nn.utils.clip_grad_norm_(m.parameters(), 20)
        assert abs(float(tn) - float(norms[k])) < 1e-3 * float(tn)
        torch.testing.assert_close(st.params["w1"].grad[k], m.linear1.weight.grad, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(st.params["b2"].grad[k], m.linear2.bias.grad, rtol=1e-5, atol=1e-6)


def test_value_stack_and_padding_stays_zero_under_adam():
    dims = [5, 8]
    mods = _mods(Value, dims, 6)
    st = StackedNets(mods, dims, "mlp", "cpu", act=None)
    opt = torch.optim.Adam(st.parameters(), lr=0.1)
    x = torch.randn(2, 9, 8)
    x[0, :, 5:] = 0
    for _ in range(3):
        opt.zero_grad()
        st.forward(x).pow(2).sum().backward()
        opt.step()
    assert torch.count_nonzero(st.params["w1"][0, :, 5:]) == 0
    assert mods[0].linear1.weight.shape == (6, 5)
