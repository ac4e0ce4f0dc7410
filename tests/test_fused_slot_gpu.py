"""The fused env + policy rollout slot (d2d_comb_policy_fused_step, env_kernels.hip
comb_policy_fused_kernel) against the two-launch slot it replaces (d2d_env_step, then d2d_policy_mlp_step:
the loop body of create_rollouts, /root/reference/algorithms/ippo.py:293-330, whose parity with the reference
the learner and env tests establish).  Bar: bit-exact -- the same record bytes, env state, rewards, actions
and log-probs, in sampling and deterministic mode, on a ragged env count (not a multiple of the 32- or 64-env
slice), and a whole iPPO training rollout with D2D_FUSED_SLOT on equal to the default rollout.  Oracle pin
(test_fused_slot_matches_c_oracle_and_torch_policy): the fused launch against the C oracle env and the reference
Policy in torch fp32 on the same Philox stream, not only against the two-launch HIP slot.  The row is a measured
negative result (580 vs 252 us), off the product path (D2D_FUSED_SLOT defaults to 0)."""
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _learner(E, seed=5, H=64):
    import bench
    from algorithms.ippo import iPPO
    from envs.combinatorial_env import CombinatorialEnv
    env = CombinatorialEnv(**bench.config3_params(200), n_envs=E, device="cuda:0", seed=seed)
    torch.manual_seed(3)
    return iPPO(env, hidden_size=H, gamma=0.6, policy_lr=3e-4, value_lr=1e-3, device="cuda:0", combinatorial=True)


def _state(b):
    return [t.clone() for t in (b.buffers, b.channels, b.received, b.discarded)]


@pytest.mark.parametrize("slice_envs", [32, 64])
@pytest.mark.parametrize("deterministic", [False, True], ids=["sample", "deterministic"])
@pytest.mark.parametrize("H", [64, 32])
def test_fused_slot_equals_env_step_then_policy(slice_envs, deterministic, H):
    from d2dhip import _lib
    from d2dhip.record import set_format
    lib = _lib.require_gpu()
    lib.d2d_set_option(_lib.D2D_OPT_FUSED_SLICE, slice_envs)
    try:
        _check_slots(deterministic, H, set_format)
    finally:
        lib.d2d_set_option(_lib.D2D_OPT_FUSED_SLICE, 0)


def _check_slots(deterministic, H, set_format):
    E = 1000  # ragged: 31.25 slices of 32, 15.6 of 64
    lr_a, lr_b = _learner(E, H=H), _learner(E, H=H)
    lr_b._pseed = lr_a._policy_seed()  # (drawn lazily from torch's RNG: the second learner's draw would differ)
    ba, bb = lr_a.env.batch(), lr_b.env.batch()
    recs = [b.record_buffer((2,)) for b in (ba, bb)]
    for b, rec in zip((ba, bb), recs):
        b.reset(want_obs=True, out_obs=rec[0])
    N = ba.spec.N
    acts = [[b.action_buffer() for _ in range(2)] for b in (ba, bb)]
    logps = [[torch.zeros((N, E), dtype=torch.float32, device="cuda:0") for _ in range(2)] for _ in range(2)]
    rews = [torch.zeros(E, dtype=torch.int32, device="cuda:0") for _ in range(2)]
    # slot 0's policy on both (the two-launch kernel)
    for j, (lr, b) in enumerate(((lr_a, ba), (lr_b, bb))):
        lr._policy_slot(recs[j], 0, 0, not deterministic, acts[j][0], logps[j][0], None, None, b)
    desc = lr_b._mlp_desc(E, bb.desc.env_base, critic=False)
    desc.rng_offset = bb.rng_off.data_ptr()
    set_format(desc, recs[1][0])
    for t in range(6):
        cur, nxt = t % 2, (t + 1) % 2
        # A: env step t, then the policy of slot t + 1
        ba.step(acts[0][cur], want_obs=True, out_obs=recs[0][nxt], out_reward=rews[0])
        lr_a._policy_slot(recs[0], 0, nxt, not deterministic, acts[0][nxt], logps[0][nxt], None, None, ba)
        # B: one fused launch
        bb.step_policy_fused(acts[1][cur], recs[1][nxt], rews[1], desc, deterministic, acts[1][nxt], logps[1][nxt])
        torch.cuda.synchronize()
        assert torch.equal(recs[0][nxt].data, recs[1][nxt].data), f"record, slot {t + 1}"
        assert torch.equal(rews[0], rews[1]), f"reward, slot {t}"
        for x, y in zip(_state(ba), _state(bb)):
            assert torch.equal(x, y), f"env state, slot {t}"
        assert torch.equal(acts[0][nxt], acts[1][nxt]), f"actions, slot {t + 1}"
        assert torch.equal(logps[0][nxt], logps[1][nxt]), f"log-probs, slot {t + 1}"
    assert ba.rng_step == bb.rng_step and ba.timestep == bb.timestep


def test_fused_slot_rollout_equals_default_rollout():
    """A whole 200-slot iPPO training rollout (eager and graph-captured) with the fused slots: identical
    records, actions, log-probs and rewards."""
    E = 2048
    out = []
    for fused in (False, True):
        lr = _learner_with(E, fused)
        ro = lr._rollout(E, defer_values=True)
        ro2 = lr._rollout(E, defer_values=True)  # the second rollout replays the captured graph
        torch.cuda.synchronize()
        out.append([(r.obs.data.clone(), r.actions.clone(), r.logp.clone(), r.rewards.clone()) for r in (ro, ro2)])
    for k in range(2):
        for x, y, name in zip(out[0][k], out[1][k], ("record", "actions", "logp", "rewards")):
            assert torch.equal(x, y), f"rollout {k}: {name}"


def _learner_with(E, fused):
    lr = _learner(E)
    lr.fused_slot = fused
    assert lr._fused_ok()
    return lr


def test_fused_slot_refuses_outside_prototype_scope():
    from d2dhip import _lib
    _lib.require_gpu()
    lr = _learner(64, H=128)
    b = lr.env.batch()
    rec = b.record_buffer((1,))
    b.reset(want_obs=True, out_obs=rec[0])
    from d2dhip.record import set_format
    desc = lr._mlp_desc(64, b.desc.env_base, critic=False)
    set_format(desc, rec[0])
    act, act2 = b.action_buffer(), b.action_buffer()
    logp = torch.zeros((64, 64), dtype=torch.float32, device="cuda:0")
    with pytest.raises(NotImplementedError, match="hidden <= 64"):
        b.step_policy_fused(act, rec[0], None, desc, False, act2, logp)
    lr64 = _learner(64, H=64)
    b64 = lr64.env.batch()
    rec64 = b64.record_buffer((1,))
    b64.reset(want_obs=True, out_obs=rec64[0])
    desc2 = lr64._mlp_desc(64, b64.desc.env_base, critic=True)  # with the critic
    set_format(desc2, rec64[0])
    with pytest.raises(NotImplementedError, match="no critic"):
        b64.step_policy_fused(b64.action_buffer(), rec64[0], None, desc2, False, b64.action_buffer(), logp)
    with pytest.raises(ValueError, match="obs_record"):  # an fp32-row output
        b64.step_policy_fused(b64.action_buffer(), b64.obs, None, desc2, False, b64.action_buffer(), logp)


def _policy_probs_fp32(pp, obs):
    """The reference Policy (ippo.py:54-71: linear1, relu, linear2, softmax) of every agent in torch fp32 on the
    oracle's obs [E][N][F]: probs [N][E][A]."""
    x = obs.transpose(0, 1)
    h = torch.relu(torch.baddbmm(pp["b1"].unsqueeze(1), x, pp["w1"].transpose(1, 2)))
    return torch.softmax(torch.baddbmm(pp["b2"].unsqueeze(1), h, pp["w2"].transpose(1, 2)), -1)


@pytest.mark.parametrize("deterministic", [False, True], ids=["sample", "deterministic"])
def test_fused_slot_matches_c_oracle_and_torch_policy(deterministic):
    """Oracle pin of the fused slot (/root/reference/algorithms/ippo.py:293-330): over 6 fused
    slots of a ragged 300-env batch, the C oracle env (oracle/c/d2d_oracle.c, the restatement of
    CombinatorialEnv.step pinned to the reference's own fixtures) stepping the same actions at the same Philox
    counters reproduces the fused launch's records (decoded obs) and rewards bit for bit; the reference Policy in
    torch fp32 (softmax -> Bernoulli, ippo.py:54-71, 154-176) on the ORACLE's obs, with the Philox uniforms of
    oracle/philox.py (stream 3 at the slot's rng_step), gives the fused launch's sampled actions (ties |u - p| <
    1e-6 excluded) or deterministic actions (p > 0.5), and its log-probs within 1e-5 wherever every probability of
    the (agent, env) lies in [1e-3, 1 - 1e-3] (1e-3 elsewhere: tests/test_policy_gpu.py's bar)."""
    import numpy as np
    import bench
    from oracle import philox
    from oracle.c_oracle import COracle
    from d2dhip.record import set_format
    from torch.distributions import Bernoulli
    E, seed = 300, 9
    lr = _learner(E, seed=seed)
    b = lr.env.batch()
    N, C = b.spec.N, b.spec.C
    c = COracle("comb", bench.config3_params(200), n_envs=E, seed=seed, env_base=int(b.desc.env_base))
    rec = b.record_buffer((2,))
    assert b.rng_step == 0
    b.reset(want_obs=True, out_obs=rec[0])
    oc = c.reset(rng_step=0, want_state=False)
    assert np.array_equal(rec[0].decode().cpu().numpy(), oc["obs"])
    pp = {k: v.data for k, v in lr.policy.params.items()}
    act = [b.action_buffer() for _ in range(2)]
    logp = [torch.zeros((N, E), dtype=torch.float32, device="cuda:0") for _ in range(2)]
    rew = torch.zeros(E, dtype=torch.int32, device="cuda:0")
    lr._policy_slot(rec, 0, 0, not deterministic, act[0], logp[0], None, None, b)  # slot 0 (no env step before it)
    desc = lr._mlp_desc(E, b.desc.env_base, critic=False)
    desc.rng_offset = b.rng_off.data_ptr()
    set_format(desc, rec[0])
    pseed = lr._policy_seed()
    envs = (int(b.desc.env_base) + np.arange(E)).astype(np.uint64)
    agents = np.arange(N, dtype=np.uint64)

    def bits_of(a):  # [E][N] uint8 masks -> [E][N][C]
        return np.unpackbits(a.cpu().numpy().view(np.uint8).reshape(E, N, -1), axis=2, bitorder="little")[:, :, :C]

    checked_sampled = 0
    for t in range(6):
        cur, nxt = t % 2, (t + 1) % 2
        rs = b.rng_step
        a_t = bits_of(act[cur])
        b.step_policy_fused(act[cur], rec[nxt], rew, desc, deterministic, act[nxt], logp[nxt])
        oc = c.step(a_t, rng_step=rs, want_state=False)
        torch.cuda.synchronize()
        assert np.array_equal(rec[nxt].decode().cpu().numpy(), oc["obs"]), f"record vs oracle obs, slot {t + 1}"
        assert np.array_equal(rew.cpu().numpy(), oc["reward"]), f"reward vs oracle, slot {t}"
        # the policy of slot t + 1 on the oracle's obs
        probs = _policy_probs_fp32(pp, torch.from_numpy(oc["obs"]).to("cuda:0"))       # [N][E][C]
        p = probs.double().cpu().numpy()
        got = bits_of(act[nxt]).transpose(1, 0, 2)                                      # [N][E][C]
        if deterministic:
            near = np.abs(p - 0.5) < 1e-6
            want = (p > 0.5).astype(np.uint8)
        else:
            r = philox.words(envs[None, :], agents[:, None], rs + 1, 3, 4 * ((C + 3) // 4), pseed)
            u = (r[..., :C] >> np.uint64(8)).astype(np.float64) / 16777216.0
            near = np.abs(u - p) < 1e-6
            want = (u < p).astype(np.uint8)
            checked_sampled += int((~near).sum())
        assert np.array_equal(np.where(near, 0, got), np.where(near, 0, want)), f"actions, slot {t + 1}"
        ref_lp = Bernoulli(probs=probs, validate_args=False).log_prob(
            torch.from_numpy(got).to("cuda:0", torch.float32)).mean(-1)
        well = ((probs > 1e-3) & (probs < 1 - 1e-3)).all(-1)
        assert well.float().mean() > 0.5
        torch.testing.assert_close(logp[nxt][well], ref_lp[well], rtol=0, atol=1e-5)
        torch.testing.assert_close(logp[nxt], ref_lp, rtol=0, atol=1e-3)
    assert deterministic or checked_sampled > 0.99 * 6 * N * E * C
