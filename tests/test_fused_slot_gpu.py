"""The fused env + policy rollout slot (d2d_comb_policy_fused_step, env_kernels.hip
comb_policy_fused_kernel) against the two-launch slot it replaces (d2d_env_step, then d2d_policy_mlp_step:
the loop body of create_rollouts, /root/reference/algorithms/ippo.py:293-330, whose parity with the reference
the learner and env tests establish).  Bar: bit-exact -- the same record bytes, env state, rewards, actions
and log-probs, in sampling and deterministic mode, on a ragged env count (not a multiple of the 32- or 64-env
slice), and a whole iPPO training rollout with D2D_FUSED_SLOT on equal to the default rollout."""
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
