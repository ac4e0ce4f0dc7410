"""World-size-2 gloo tests (CPU) of the data-parallel path (algorithms/data_parallel.py):
a learner step on two env shards with the bucketed gradient all-reduce must equal
the single-process step on the whole batch; global normalisation statistics from
shard sums equal the unsharded ones; the D2D permutation and initial weights are
identical on every rank.  Tolerance: 1e-6 absolute (fp32 summation order)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, ws, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)


def _problem(seed=0):
    from algorithms._core import Policy, StackedNets
    torch.manual_seed(seed)
    dims = [12, 9, 12]
    mods = [Policy(d, 5, 16) for d in dims]
    st = StackedNets(mods, dims, "mlp", "cpu", act="softmax")
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.randn(3, 64, 12, generator=g)
    x[1, :, 9:] = 0
    acts = (torch.rand(3, 64, 5, generator=g) < 0.3).float()
    adv = torch.randn(64, generator=g)
    logp_old = torch.randn(3, 64, generator=g) * 0.1 - 3.0
    return st, x, acts, adv, logp_old


def _d2d_epoch(st, opt, x, acts, adv, logp_old, perm, reduce_fn):
    from algorithms._core import make_dist
    from algorithms.d2d_ppo import happo_chain
    probs = st.forward(x)
    dist_ = make_dist(probs, True)
    logp = dist_.log_prob(acts).mean(-1)
    ent = dist_.entropy().mean(-1)
    ratio = torch.exp(logp - logp_old)
    M = happo_chain(adv, ratio.detach(), perm)
    loss = -torch.min(ratio * M, torch.clamp(ratio, 0.9, 1.1) * M).mean(1) - 0.01 * ent.mean(1)
    opt.zero_grad()
    loss.sum().backward()
    reduce_fn(st.parameters())
    st.grad_norm_clip_(20)
    opt.step()


def _worker(rank, ws, port, outdir):
    from algorithms import data_parallel as dp
    _init(rank, ws, port)
    try:
        st, x, acts, adv, logp_old = _problem()
        # every rank starts from rank 0's weights even if its own init differs
        if rank == 1:
            with torch.no_grad():
                for p in st.parameters():
                    p.add_(0.5)
        dp.broadcast_params_(st.parameters())
        perm = np.random.default_rng(100 + rank).permutation(3)   # ranks disagree ...
        perm = dp.broadcast_perm(perm, "cpu")                     # ... until the broadcast
        B = x.shape[1] // ws
        sl = slice(rank * B, (rank + 1) * B)
        # NB: the happo chain's advantage is already globally normalised; shard it like the samples
        opt = torch.optim.Adam(st.parameters(), lr=1e-2)
        for _ in range(2):
            _d2d_epoch(st, opt, x[:, sl], acts[:, sl], adv[sl], logp_old[:, sl], perm, dp.allreduce_grads_)
        torch.save({k: v.detach().clone() for k, v in st.params.items()}, os.path.join(outdir, f"w{rank}.pt"))
        np.save(os.path.join(outdir, f"perm{rank}.npy"), perm)
        # global column statistics from shard-local sums
        rng = np.random.default_rng(7)
        full = torch.from_numpy(rng.normal(size=(1000, 4)) * [1, 2, 3, 4] + [0, 1, 2, 3])
        loc = full[rank * 500:(rank + 1) * 500]
        mean, std = dp.combine_column_stats(loc.sum(0), lambda m: ((loc - m) ** 2).sum(0), 500, 1)
        np.save(os.path.join(outdir, f"stats{rank}.npy"), torch.stack([mean, std]).numpy())
    finally:
        dist.destroy_process_group()


def test_two_rank_update_equals_full_batch(tmp_path):
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    # single-process reference on the full batch
    st, x, acts, adv, logp_old = _problem()
    perm = np.load(tmp_path / "perm0.npy")
    assert np.array_equal(perm, np.load(tmp_path / "perm1.npy"))
    opt = torch.optim.Adam(st.parameters(), lr=1e-2)
    for _ in range(2):
        _d2d_epoch(st, opt, x, acts, adv, logp_old, perm, lambda ps: None)
    w0 = torch.load(tmp_path / "w0.pt")
    w1 = torch.load(tmp_path / "w1.pt")
    for k, v in st.params.items():
        torch.testing.assert_close(w0[k], w1[k], rtol=0, atol=0)
        torch.testing.assert_close(w0[k], v.detach(), rtol=0, atol=1e-6)
    s0, s1 = np.load(tmp_path / "stats0.npy"), np.load(tmp_path / "stats1.npy")
    rng = np.random.default_rng(7)
    full = rng.normal(size=(1000, 4)) * [1, 2, 3, 4] + [0, 1, 2, 3]
    np.testing.assert_allclose(s0, s1, rtol=0, atol=0)
    np.testing.assert_allclose(s0[0], full.mean(0), rtol=0, atol=1e-12)
    np.testing.assert_allclose(s0[1], full.std(0, ddof=1), rtol=0, atol=1e-12)


def test_single_process_hooks_are_identity():
    from algorithms.data_parallel import DataParallelMixin, world
    assert world() == (0, 1)

    class L(DataParallelMixin):
        pass

    lr = L()
    assert lr._last_shard() and lr._n_envs_total() is None
    assert list(lr._sync_perm(np.array([2, 0, 1]))) == [2, 0, 1]
