"""d2d_f32_to_bf16_exact (ABI v7): the D2D central critic's bf16 state operand, converted and checked for
bf16-exactness in one pass (algorithms/d2d_ppo.py _critic_split_forward; the states of the reference's
central Value net, d2d_ppo.py:95-98, are small integers)."""
import pytest
import torch

from d2dhip import _lib

pytestmark = pytest.mark.gpu


def run(x):
    lib = _lib.require_gpu()
    out = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    flag = torch.full((1,), 7, dtype=torch.int32, device=x.device)
    _lib.check(lib.d2d_f32_to_bf16_exact(x.numel(), x.data_ptr(), out.data_ptr(), flag.data_ptr(), _lib.stream_ptr()),
               "d2d_f32_to_bf16_exact")
    torch.cuda.synchronize()
    return out, int(flag.item())


@pytest.mark.parametrize("n", [0, 1, 3, 4, 5, 1023, 4096 * 15 + 7, 3 * (1 << 20) + 2])
def test_integer_states_are_exact(n):
    g = torch.Generator(device="cuda").manual_seed(n)
    x = torch.randint(-128, 256, (n,), device="cuda", generator=g).float()
    out, flag = run(x)
    assert flag == 0
    assert torch.equal(out, x.to(torch.bfloat16))
    assert torch.equal(out.float(), x)


@pytest.mark.parametrize("pos", [0, 1, 2, 3, 4, 777, -1])
def test_one_inexact_value_is_flagged(pos):
    n = 10_003
    x = torch.randint(0, 8, (n,), device="cuda").float()
    x[pos] = 1.0 + 2.0 ** -10  # not representable in bf16 (8 significand bits)
    out, flag = run(x)
    assert flag == 1
    keep = torch.ones(n, dtype=torch.bool, device="cuda")
    keep[pos] = False
    assert torch.equal(out[keep].float(), x[keep])
    assert out[pos].float().item() == 1.0  # the high half (truncation)


def test_2d_state_batch_matches_torch_conversion():
    x = torch.randint(0, 15, (4096, 3848), device="cuda").float()  # S = 15 N + 8 at 256 agents
    x[:, -8:] = torch.randint(-1, 2, (4096, 8), device="cuda").float()
    out, flag = run(x)
    assert flag == 0 and torch.equal(out, x.to(torch.bfloat16))


def test_rejects_misaligned_input():
    x = torch.zeros(65, device="cuda")
    out = torch.empty(64, dtype=torch.bfloat16, device="cuda")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    rc = _lib.require_gpu().d2d_f32_to_bf16_exact(64, x.data_ptr() + 4, out.data_ptr(), flag.data_ptr(),
                                                   _lib.stream_ptr())
    assert rc != 0


@pytest.mark.parametrize("T,E,S,ld", [(200, 64, 3848, 3848), (7, 5, 23, 24), (3, 2, 3848, 3852), (200, 33, 21, 21)])
def test_states_from_the_slot_major_buffer(T, E, S, ld):
    """d2d_states_to_bf16_exact: the env-major operand [E*T][S] straight from the rollout buffer [T][E][ld]."""
    g = torch.Generator(device="cuda").manual_seed(T + E + S)
    x = torch.randint(-1, 20, (T, E, ld), device="cuda", generator=g).float()
    ref = x[:, :, :S].transpose(0, 1).reshape(E * T, S)
    out = torch.empty((E * T, S), dtype=torch.bfloat16, device="cuda")
    flag = torch.full((1,), 7, dtype=torch.int32, device="cuda")
    lib = _lib.require_gpu()
    _lib.check(lib.d2d_states_to_bf16_exact(T, E, S, ld, x.data_ptr(), out.data_ptr(), flag.data_ptr(),
                                            _lib.stream_ptr()), "d2d_states_to_bf16_exact")
    torch.cuda.synchronize()
    assert int(flag.item()) == 0 and torch.equal(out, ref.to(torch.bfloat16))
    x[T - 1, E - 1, S - 1] = 0.3  # one inexact state value (padding columns past S are not read)
    x[0, 0, ld - 1] = 0.3 if ld > S else x[0, 0, ld - 1]
    _lib.check(lib.d2d_states_to_bf16_exact(T, E, S, ld, x.data_ptr(), out.data_ptr(), flag.data_ptr(),
                                            _lib.stream_ptr()), "d2d_states_to_bf16_exact")
    torch.cuda.synchronize()
    assert int(flag.item()) == 1


@pytest.mark.parametrize("T,E,S,ld,out_ld", [(200, 64, 117, 117, 120), (7, 5, 23, 24, 24), (3, 2, 128, 132, 136),
                                             (20, 33, 248, 248, 248)])
def test_states_padded_rows(T, E, S, ld, out_ld):
    """d2d_states_to_bf16_padded (ABI v10): rows of out_ld bf16, the states in [0, S) and zeros in [S, out_ld)
    (the pad columns are overwritten whatever the buffer held)."""
    g = torch.Generator(device="cuda").manual_seed(T + E + S)
    x = torch.randint(-1, 20, (T, E, ld), device="cuda", generator=g).float()
    ref = torch.zeros((E * T, out_ld), device="cuda")
    ref[:, :S] = x[:, :, :S].transpose(0, 1).reshape(E * T, S)
    out = torch.full((E * T, out_ld), 5.0, dtype=torch.bfloat16, device="cuda")
    flag = torch.full((1,), 7, dtype=torch.int32, device="cuda")
    lib = _lib.require_gpu()
    _lib.check(lib.d2d_states_to_bf16_padded(T, E, S, ld, x.data_ptr(), out.data_ptr(), out_ld, flag.data_ptr(),
                                             _lib.stream_ptr()), "d2d_states_to_bf16_padded")
    torch.cuda.synchronize()
    assert int(flag.item()) == 0 and torch.equal(out, ref.to(torch.bfloat16))
    assert lib.d2d_states_to_bf16_padded(T, E, S, ld, x.data_ptr(), out.data_ptr(), S - 1, flag.data_ptr(),
                                         _lib.stream_ptr()) == -1  # D2D_EINVAL
