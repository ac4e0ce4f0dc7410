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
        # global column statistics: the product's cross-rank protocol (d2dhip.gae.two_pass_column_stats,
        # the one normalize_columns_ runs between its HIP kernels) driven with the oracle's arithmetic
        from d2dhip.gae import two_pass_column_stats
        from oracle.gae_oracle import colstats_finalize
        rng = np.random.default_rng(7)
        full = torch.from_numpy(rng.normal(size=(1000, 4)) * [1, 2, 3, 4] + [0, 1, 2, 3])
        loc = full[rank * 500:(rank + 1) * 500]
        for ddof in (0, 1):
            mean, scale, gate = two_pass_column_stats(
                lambda c: (loc.sum(0) if c is None else ((loc - c) ** 2).sum(0)).clone(),
                lambda s1, m2: colstats_finalize(s1, m2, 1000.0, ddof), dp.dist.group.WORLD)
            np.save(os.path.join(outdir, f"stats{rank}_{ddof}.npy"),
                    torch.stack([mean, 1.0 / scale, gate.double().expand(4)]).numpy())
            # the same statistics from the scan's fused per-rank moments (n, sum, M2 about the local mean;
            # d2d_gae_scan_moments) through gae.moments_colsum: no second pass over the data
            from d2dhip.gae import moments_colsum
            mom = torch.stack([torch.full((4,), 500.0, dtype=torch.float64), loc.sum(0),
                               ((loc - loc.mean(0)) ** 2).sum(0)])
            mean, scale, gate = two_pass_column_stats(moments_colsum(mom, True),
                                                      lambda s1, m2: colstats_finalize(s1, m2, 1000.0, ddof),
                                                      dp.dist.group.WORLD)
            np.save(os.path.join(outdir, f"mstats{rank}_{ddof}.npy"),
                    torch.stack([mean, 1.0 / scale, gate.double().expand(4)]).numpy())
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
    rng = np.random.default_rng(7)
    full = rng.normal(size=(1000, 4)) * [1, 2, 3, 4] + [0, 1, 2, 3]
    for ddof in (0, 1):
        s0, s1 = np.load(tmp_path / f"stats0_{ddof}.npy"), np.load(tmp_path / f"stats1_{ddof}.npy")
        np.testing.assert_allclose(s0, s1, rtol=0, atol=0)
        np.testing.assert_allclose(s0[0], full.mean(0), rtol=0, atol=1e-12)
        np.testing.assert_allclose(s0[1], full.std(0, ddof=ddof), rtol=0, atol=1e-12)
        assert np.all(s0[2] == 1)
        m0, m1 = np.load(tmp_path / f"mstats0_{ddof}.npy"), np.load(tmp_path / f"mstats1_{ddof}.npy")
        np.testing.assert_allclose(m0, m1, rtol=0, atol=0)
        np.testing.assert_allclose(m0, s0, rtol=0, atol=1e-12)


def test_single_process_hooks_are_identity():
    from algorithms.data_parallel import DataParallelMixin, world
    assert world() == (0, 1)

    class L(DataParallelMixin):
        pass

    lr = L()
    assert lr._last_shard() and lr._n_envs_total() is None
    assert list(lr._sync_perm(np.array([2, 0, 1]))) == [2, 0, 1]


class _StubEnv:  # noqa: E302
    """Just the env attributes DataParallelMixin._setup_data_parallel reads (no GPU needed)."""

    def __init__(self, n_envs, batch_env_base=None):
        from types import SimpleNamespace
        self.n_envs = n_envs
        self.env_base = 0
        self._batch = None if batch_env_base is None else SimpleNamespace(desc=SimpleNamespace(env_base=batch_env_base))

    def shard(self, rank, world_size):
        self.env_base = rank * self.n_envs
        return self


def _shard_worker(rank, ws, port, outdir):
    from algorithms.data_parallel import DataParallelMixin

    class L(DataParallelMixin):
        pass

    _init(rank, ws, port)
    try:
        res = []
        # (a) env batch not built yet: the learner shards it
        lr = L()
        lr.env = _StubEnv(8)
        lr._setup_data_parallel([torch.zeros(3)])
        res.append(lr.env.env_base)
        # (b) env batch built before the learner with the default env_base 0: rank 0 is fine,
        # every other rank must refuse (identical Philox streams on all ranks otherwise)
        lr = L()
        lr.env = _StubEnv(8, batch_env_base=0)
        try:
            lr._setup_data_parallel([torch.zeros(3)])
            res.append("ok")
        except RuntimeError:
            res.append("refused")
        np.save(os.path.join(outdir, f"shard{rank}.npy"), np.array([str(r) for r in res]))
    finally:
        dist.destroy_process_group()


def test_data_parallel_refuses_unsharded_env(tmp_path):
    port = _free_port()
    mp.spawn(_shard_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    # rank 1's batch draws rank 0's streams; both ranks refuse (collectively, nobody hangs)
    assert list(np.load(tmp_path / "shard0.npy")) == ["0", "refused"]
    assert list(np.load(tmp_path / "shard1.npy")) == ["8", "refused"]
