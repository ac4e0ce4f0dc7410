"""d2d_env_out.state_bf16 (ABI v13): the combinatorial env kernel writes D2D-PPO's state rows (combinatorial_env.py:
207-209) as the central critic's bf16 operand -- exact, every state value is an integer in [-1, 255] -- straight into
an env-major [E][T][S8] rollout buffer.  Bars: bit-exact against the fp32 state rows of the same step (one wave per env,
N <= 64, and the LARGE one-env-per-workgroup path, N > 64), the pad columns zero, the rows of other slots untouched;
and a D2D-PPO training iteration on the bf16 rows equal to one on the fp32 rows + the conversion pass."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.mark.parametrize("N,C,E", [(6, 3, 37), (64, 8, 100), (96, 8, 20), (256, 8, 9)])
def test_state_bf16_rows_equal_fp32_rows(N, C, E):
    from d2dhip.envbatch import EnvBatch
    from envs.combinatorial_env import CombinatorialEnv
    env = CombinatorialEnv(N, C, np.resize(np.array([3, 7, 14]), N), np.full(N, 0.4), episode_length=20,
                           channel_switch=np.full((N, C), 0.3), n_envs=E, device="cuda", seed=11)
    b = env.batch()
    assert isinstance(b, EnvBatch)
    s = b.spec
    S8 = -(-s.S // 8) * 8
    T = 5
    xb = torch.full((E, T, S8 + 8), 7.0, dtype=torch.bfloat16, device="cuda")  # extra columns: must stay untouched
    st = torch.zeros((E, s.state_stride), dtype=torch.float32, device="cuda")
    b.reset(want_obs=False, out_state=st, out_state_bf16=xb[:, 0])
    ref = [st[:, : s.S].clone()]
    act = b.action_buffer()
    for t in range(1, T):
        b.sample_actions(0.3, out=act)
        b.step(act, want_obs=False, out_state=st, out_state_bf16=xb[:, t])
        ref.append(st[:, : s.S].clone())
    torch.cuda.synchronize()
    for t in range(T):
        assert torch.equal(xb[:, t, : s.S].float(), ref[t]), f"slot {t}"
        assert torch.all(xb[:, t, s.S:S8] == 0), f"pad, slot {t}"
        assert torch.all(xb[:, t, S8:] == 7.0), f"past the row, slot {t}"
    assert float(ref[-1].abs().max()) > 1  # packet counts, not only bits


def test_state_bf16_argument_checks():
    from envs.channel_selection_env import ChannelSelectionEnv
    from envs.combinatorial_env import CombinatorialEnv
    env = CombinatorialEnv(6, 3, np.full(6, 5), np.full(6, 0.3), episode_length=10, channel_switch=np.full((6, 3), 0.3),
                           n_envs=8, device="cuda", seed=1)
    b = env.batch()
    with pytest.raises(ValueError):  # too narrow
        b.reset(want_obs=False, out_state_bf16=torch.zeros((8, 8), dtype=torch.bfloat16, device="cuda"))
    with pytest.raises(ValueError):  # row stride not a multiple of 8
        x = torch.zeros((8, 61), dtype=torch.bfloat16, device="cuda")[:, :56]
        b.reset(want_obs=False, out_state_bf16=x)
    ch = ChannelSelectionEnv(6, 3, np.full(6, 5), np.full(6, 0.3), episode_length=10, channel_switch=np.full(4, 0.3),
                             n_envs=8, device="cuda", seed=1)
    with pytest.raises(NotImplementedError):
        ch.batch().reset(want_obs=False, out_state_bf16=torch.zeros((8, 64), dtype=torch.bfloat16, device="cuda"))


@pytest.mark.parametrize("N", [16, 96])
def test_d2d_iteration_on_bf16_state_rows_equals_fp32_states(N, monkeypatch):
    """One rollout + two update epochs of D2D-PPO (MLP, combinatorial) with the env kernel's bf16 state rows and
    with fp32 states + d2d_states_to_bf16_padded: the same states, values, losses and weights, bit for bit."""
    from algorithms.d2d_ppo import D2DPPO
    from envs.combinatorial_env import CombinatorialEnv
    out = []
    for bf in (False, True):
        monkeypatch.setattr(D2DPPO, "state_bf16_rollout", bf)
        env = CombinatorialEnv(N, 8, np.full(N, 7), np.full(N, 1 / 14), episode_length=30,
                               channel_switch=np.full((N, 8), 0.8), n_envs=64, device="cuda", seed=5)
        torch.manual_seed(2)
        np.random.seed(2)
        lr = D2DPPO(env, hidden_size=64, gamma=0.4, device="cuda", combinatorial=True, early_stopping=False)
        ro = lr._rollout(64)
        assert (ro.__dict__.get("states") is None) == bf
        upd = lr._update_state(ro)
        losses = [lr._update_epoch(ro, upd) for _ in range(2)]
        torch.cuda.synchronize()
        out.append((ro.state_seq.clone(), [float(v) for _, v in losses],
                    [p.detach().clone() for p in lr.value_network.parameters()],
                    [p.detach().clone() for p in lr.policy.parameters()]))
    assert torch.equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1]
    for a, b in zip(out[0][2] + out[0][3], out[1][2] + out[1][3]):
        assert torch.equal(a, b)
