"""Host logic of the learners' Rollout record (algorithms/_learner.py): the env-major views the
reference's sample order needs (d2d_ppo.py:333-339 concatenates episodes env by env) are derived
lazily from the slot-major device buffers, on CPU tensors here."""
import torch

from algorithms._learner import Rollout


def test_state_seq_is_the_env_major_view_of_the_state_buffer():
    T, E, stride, S = 5, 3, 8, 6
    states = torch.arange(T * E * stride, dtype=torch.float32).reshape(T, E, stride)
    ro = Rollout(states=states, state_dim=S)
    assert "state_seq" not in ro.__dict__  # nothing materialised until asked
    seq = ro.state_seq
    assert seq.shape == (E * T, S)
    for e in range(E):
        for t in range(T):
            assert torch.equal(seq[e * T + t], states[t, e, :S])
    assert ro.state_seq is seq  # cached


def test_state_seq_set_explicitly_wins():
    s = torch.zeros(4, 2)
    ro = Rollout(states=torch.ones(2, 2, 3), state_dim=2, state_seq=s)
    assert ro.state_seq is s


def test_adv_ret_views_from_the_gae_layout():
    T, N, E = 4, 2, 3
    adv_tne = torch.arange(T * N * E, dtype=torch.float32).reshape(T, N, E)
    ro = Rollout(adv_tne=adv_tne)
    adv = ro.adv  # agent-major [N][E*T], env-major sample order
    assert adv.shape == (N, E * T)
    for k in range(N):
        for e in range(E):
            for t in range(T):
                assert adv[k, e * T + t] == adv_tne[t, k, e]
