"""CPU-side checks of the drop-in boundary: the C-ABI library loads and exports
every symbol include/d2d_hip.h declares (no compute calls without a GPU), the
ctypes structs match the header layout, and the host logic (spec derivation,
mask packing, reference-API attributes) behaves like the reference."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "d2d_hip.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(d2d_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    import d2dhip
    lib = d2dhip.load()
    fns = header_functions()
    assert len(fns) >= 12
    for fn in fns:
        assert hasattr(lib, fn), fn
        assert fn in d2dhip.EXPORTED, f"{fn} has no ctypes signature"
    assert lib.d2d_abi_version() == 15
    assert [lib.d2d_mask_bytes(c) for c in (1, 8, 9, 16, 17, 32)] == [1, 1, 2, 2, 4, 4]
    assert [lib.d2d_buffer_words(d) for d in (1, 4, 5, 8, 12, 14, 16, 17, 32)] == [1, 1, 2, 2, 3, 4, 4, 8, 8]
    assert lib.d2d_colstats_workspace(1000, 64) >= 64


def test_ctypes_structs_match_header_layout():
    from d2dhip import _lib
    from d2dhip.spec import AGENT_DTYPE
    assert AGENT_DTYPE.itemsize == 32
    assert ctypes.sizeof(_lib.EnvDesc) == 8 * 4 + 8 * 2 + 8 * 8
    assert ctypes.sizeof(_lib.MlpDesc) == 6 * 4 + 8 * 8 + 8 * 2 + 8 + 2 * 4 + 8
    assert ctypes.sizeof(_lib.EnvState) == 6 * 8 and ctypes.sizeof(_lib.EnvOut) == 8 * 8  # + state_bf16, its ld (v13)
    assert ctypes.sizeof(_lib.EnvReplay) == 2 * 8
    assert ctypes.sizeof(_lib.GruDesc) == 8 * 4 + 8 * 8 + 8 * 2 + 8 + 2 * 4 + 8
    # D2D_RECORD_BYTES(obs_dim) of the header and its Python mirror
    txt = open(HEADER).read()
    assert "#define D2D_RECORD_BYTES(obs_dim) (32 * (((obs_dim) + 32) / 32))" in txt
    assert [_lib.record_bytes(f) for f in (1, 30, 31, 32, 63, 64)] == [32, 32, 32, 64, 64, 96]


def test_library_validates_arguments_without_gpu():
    """Argument checks run before any HIP call, so they work on a GPU-less host."""
    import d2dhip
    from d2dhip import _lib
    lib = d2dhip.load()
    rc = lib.d2d_env_step(None, None, None, None, None, 1, 0, None)
    assert rc == -1 and b"desc" in lib.d2d_last_error()
    desc = _lib.EnvDesc(0, 2000, 8, 7, 23, 0, 0, 1, 0, 0, None, None, None, None, None, None, None, None)
    assert lib.d2d_env_reset(ctypes.byref(desc), None, None, None, 0, None) == -2
    assert lib.d2d_gae_scan(10, 1, 0, 1, None, None, None, 0.9, 0.97, 1, None, None, None) == -1
    # obs_format checks (before any HIP call)
    w = ctypes.c_void_p(16)
    md = _lib.MlpDesc(4, 32, 30, 64, 8, 0, w, w, w, w, None, None, None, None, 0, 0, None, 7, 0, None)
    assert lib.d2d_policy_mlp_step(ctypes.byref(md), w, None, 0, 0, w, w, None, None) == -1
    assert b"obs_format" in lib.d2d_last_error()
    md.obs_format = _lib.D2D_OBS_U8
    assert lib.d2d_policy_mlp_step(ctypes.byref(md), w, None, 0, 0, w, w, None, None) == -1
    assert b"obs_signed" in lib.d2d_last_error()
    md.obs_signed = w
    assert lib.d2d_policy_mlp_step(ctypes.byref(md), ctypes.c_void_p(24), None, 0, 0, w, w, None, None) == -1
    assert b"aligned" in lib.d2d_last_error()
    # ABI 15: actions may be NULL in forced mode only
    assert lib.d2d_policy_mlp_step(ctypes.byref(md), w, None, 0, 0, None, w, None, None) == -1
    assert b"NULL" in lib.d2d_last_error()
    # the record is a combinatorial-env output only
    dsc = _lib.EnvDesc(1, 4, 3, 7, 11, 0, 0, 1, 0, 0, w, w, w, w, w, None, None, w)
    st = _lib.EnvState(w, w, w, w, w, w)
    out = _lib.EnvOut(None, None, None, None, None, 16)
    assert lib.d2d_env_reset(ctypes.byref(dsc), ctypes.byref(st), None, ctypes.byref(out), 0, None) == -2
    assert b"obs_record" in lib.d2d_last_error()
    # ABI v13: bf16 state rows (combinatorial env only, 16-byte aligned rows of >= round_up(S, 8) elements)
    out_b = _lib.EnvOut(None, None, None, None, None, None, 16, 64)
    assert lib.d2d_env_reset(ctypes.byref(dsc), ctypes.byref(st), None, ctypes.byref(out_b), 0, None) == -2
    assert b"state_bf16" in lib.d2d_last_error()
    # (the host-side tables are read on the host by argument-checked calls that pass: real arrays)
    kinds, period, offs = np.zeros(64, np.uint8), np.ones(64), np.zeros(64)
    comb = _lib.EnvDesc(0, 64, 8, 14, 30, 100, 100, 1, 0, 0, w, w, kinds.ctypes.data, period.ctypes.data,
                        offs.ctypes.data, None, None, w)
    for ptr, ld in ((16, 100), (24, 104), (16, 96)):  # ld not a multiple of 8, misaligned, narrower than 104
        bad = _lib.EnvOut(None, None, None, None, None, None, ptr, ld)
        assert lib.d2d_env_reset(ctypes.byref(comb), ctypes.byref(st), None, ctypes.byref(bad), 0, None) == -1
        assert b"state_bf16" in lib.d2d_last_error()
    # ABI v13: the fused env + policy slot's scope checks (before any HIP call)
    rec_out = _lib.EnvOut(None, None, None, None, None, 16)
    pol = _lib.MlpDesc(64, 1, 30, 64, 8, 0, w, w, w, w, None, None, None, None, 0, 0, None, _lib.D2D_OBS_U8, 0, w)
    args = (1, 0, ctypes.byref(pol), 0, 0, w, w, None)
    assert lib.d2d_comb_policy_fused_step(ctypes.byref(dsc), ctypes.byref(st), w, ctypes.byref(rec_out), *args) == -2
    assert b"combinatorial" in lib.d2d_last_error()
    rows_out = _lib.EnvOut(16, None, None, None, None, None)  # fp32 obs rows instead of the record
    assert lib.d2d_comb_policy_fused_step(ctypes.byref(comb), ctypes.byref(st), w, ctypes.byref(rows_out), *args) == -1
    assert b"obs_record" in lib.d2d_last_error()
    pol.hidden = 128
    assert lib.d2d_comb_policy_fused_step(ctypes.byref(comb), ctypes.byref(st), w, ctypes.byref(rec_out), *args) == -2
    assert b"hidden <= 64" in lib.d2d_last_error()
    pol.hidden, pol.n_envs = 64, 2
    assert lib.d2d_comb_policy_fused_step(ctypes.byref(comb), ctypes.byref(st), w, ctypes.byref(rec_out), *args) == -1
    assert b"same agents, envs" in lib.d2d_last_error()
    assert lib.d2d_set_option(_lib.D2D_OPT_FUSED_SLICE, 48) == -1
    assert lib.d2d_set_option(_lib.D2D_OPT_FUSED_SLICE, 0) == 0


def test_abi14_argument_checks():
    """ABI 14's entry points refuse bad arguments before any HIP call (runs on a GPU-less host): the carried GRU
    state (d2d_policy_gru_carry: a NULL scratch, a slot whose window does not extend the previous one) and the
    central critic's dW1 (d2d_central_critic_dw1: hidden, ldx, alignment, workspace size)."""
    import ctypes
    import d2dhip
    from d2dhip import _lib
    lib = d2dhip.load()
    w = ctypes.c_void_p(16)
    g = _lib.GruDesc(2, 32, 12, 16, 4, 1, 3, 8, w, w, w, w, w, w, w, w, 0, 0, None, _lib.D2D_OBS_F32, 0, None)
    n = lib.d2d_gru_carry_floats(ctypes.byref(g))
    assert n == 2 * 2 * 4 * 1 * 64  # [N][env tiles][4 HT][64]
    assert lib.d2d_policy_gru_carry(ctypes.byref(g), 8, w, 1, None, 0, 0, w, w, None, 1, None) == -1
    assert b"NULL hcarry" in lib.d2d_last_error()
    for slot in (0, 3, 8, 11):  # episode positions 0, 3, 0, 3 with history_len 3
        assert lib.d2d_policy_gru_carry(ctypes.byref(g), 16, w, slot, None, 0, 0, w, w, w, 1, None) == -1
        assert b"does not extend" in lib.d2d_last_error()
    assert lib.d2d_central_critic_dw1_workspace(62, 10, 100, 104) == -1
    assert lib.d2d_central_critic_dw1_workspace(64, 10, 100, 96) == -1
    ws = lib.d2d_central_critic_dw1_workspace(64, 819200, 3848, 3848)
    assert ws > 0 and ws % (64 * 3848) == 0 and (ws // (64 * 3848)) % 8 == 0  # KS partials, a multiple of the 8 XCDs
    assert lib.d2d_central_critic_dw1(62, 64, 100, 104, w, w, w, 10 ** 6, w, None) == -2
    assert lib.d2d_central_critic_dw1(64, 64, 100, 100, w, w, w, 10 ** 6, w, None) == -1  # ldx not a multiple of 8
    assert lib.d2d_central_critic_dw1(64, 64, 100, 104, ctypes.c_void_p(24), w, w, 10 ** 6, w, None) == -1  # misaligned
    assert lib.d2d_central_critic_dw1(64, 64, 100, 104, w, w, w, 1, w, None) == -1  # workspace too small
    assert b"d2d_central_critic_dw1_workspace" in lib.d2d_last_error()


def test_d2denv_record_signed_masks():
    """The D2DEnv's record masks (ABI 14): exactly the last-feedback column of each agent's obs row (gather code -1
    of d2d_env_single_gather_map, env.py:94), wherever the neighbourhood puts it."""
    import d2dhip
    from d2dhip.record import signed_masks
    from d2dhip.spec import EnvSpec
    from envs.env import D2DEnv
    lib = d2dhip.load()
    N = 5
    nb = [[0, 1], [1], [0, 1, 2, 3, 4], [3, 4], [4]]
    env = D2DEnv(n_agents=N, deadlines=np.array([3, 5, 4, 2, 6]), lbdas=np.full(N, 0.2), episode_length=10,
                 neighbourhoods=nb, n_envs=2, device="cpu", seed=1)
    s = env.spec
    codes = s.gather_map(lib)
    m = signed_masks(s, codes)
    assert m.shape == (N, 32 * ((s.F + 32) // 32) // 32)
    for k in range(N):
        cols = [c for c in range(32 * m.shape[1]) if (int(m[k, c // 32]) >> (c % 32)) & 1]
        length = sum(int(s.d[j]) + 1 for j in nb[k]) + 1  # buffers + channel bits of the neighbours, then the ack
        assert cols == [length - 1], (k, cols)
    with pytest.raises(ValueError):
        signed_masks(s)  # the D2DEnv masks need its gather codes


def test_record_signed_masks_and_decode():
    """The int8-column masks mark exactly the ACK columns [w_k + C, w_k + 2C) of every agent's row
    (combinatorial_env.py:199-206), and ObsRecord.decode maps bytes back to the fp32 obs values."""
    import torch
    from d2dhip.record import ObsRecord, signed_masks
    from d2dhip.spec import EnvSpec
    d = [7, 14, 3, 14]
    for homog, C in ((True, 8), (False, 8), (False, 16)):
        s = EnvSpec("comb", 4, C, d, [0.5] * 4, 2, [1] * 4, [0] * 4, 10, "aperiodic", [], homog, None)
        m = signed_masks(s)
        R = 32 * ((s.F + 32) // 32)
        assert m.shape == (4, R // 32) and m.dtype == np.uint32
        for k in range(4):
            cols = [c for c in range(R) if (int(m[k, c // 32]) >> (c % 32)) & 1]
            assert cols == list(range(int(s.w[k]) + C, int(s.w[k]) + 2 * C))
        rng = np.random.default_rng(C)
        obs = np.zeros((3, 4, s.F), dtype=np.float32)
        for k in range(4):
            w = int(s.w[k])
            obs[:, k, :w] = rng.integers(0, 256, size=(3, w))
            obs[:, k, w:w + C] = rng.integers(0, 2, size=(3, C))
            obs[:, k, w + C:w + 2 * C] = rng.integers(-1, 2, size=(3, C))
        raw = np.zeros((3, 4, R), dtype=np.uint8)
        raw[..., : s.F] = obs.astype(np.int16).astype(np.uint8)
        rec = ObsRecord(torch.from_numpy(raw), s.F, torch.from_numpy(m.view(np.int32)))
        assert rec.shape == (3, 4, s.F)
        assert torch.equal(rec.decode(), torch.from_numpy(obs))
        assert torch.equal(rec[1:].decode(), torch.from_numpy(obs[1:]))


def test_gpu_required_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("host has a GPU")
    from envs.combinatorial_env import CombinatorialEnv
    import d2dhip
    e = CombinatorialEnv(2, 2, np.array([3, 3]), np.ones(2))
    with pytest.raises(d2dhip.D2DHipError, match="no CPU fallback"):
        e.reset()


def test_spec_matches_reference_spaces():
    from envs.channel_selection_env import ChannelSelectionEnv
    from envs.combinatorial_env import CombinatorialEnv
    d = np.array([7, 14] * 3)
    e = CombinatorialEnv(6, 8, d, np.ones(6) * 0.5, homogeneous_size=True)
    assert [s.shape[0] for s in e.observation_space] == [30] * 6            # combinatorial_env.py:52-53
    assert e.state_space.shape == (int(d.sum()) + 8 * 7,)                   # :57-58
    assert [s.n for s in e.action_space] == [8] * 6
    e2 = CombinatorialEnv(6, 8, d, np.ones(6) * 0.5)
    assert [s.shape[0] for s in e2.observation_space] == list(d + 16)       # :49-50
    assert np.array_equal(e2.spec.obs_len, d + 16) and e2.spec.F == 30
    c = ChannelSelectionEnv(5, 16, np.array([7] * 5), np.ones(5), channel_switch=np.full(17, 0.8))
    assert [s.n for s in c.action_space] == [17] * 5                         # channel_selection_env.py:43
    assert c.state_space.shape == (35 + 17,)
    assert c.spec.F == 7 + 17


def test_spec_traffic_models_and_errors():
    from d2dhip.spec import EnvSpec, POISSON, SCHEDULED
    mk = lambda tm, pdev=(): EnvSpec("comb", 4, 2, [3, 3, 3, 3], [0.5] * 4, 2, [1] * 4, [0] * 4, 10, tm, pdev,  # noqa
                                     False, None)
    assert list(mk("aperiodic").arrival_kinds()) == [POISSON] * 4
    assert list(mk("periodic").arrival_kinds()) == [SCHEDULED] * 4
    assert list(mk("heterogeneous", np.array([1, 3])).arrival_kinds()) == [POISSON, SCHEDULED, POISSON, SCHEDULED]
    with pytest.raises(ValueError, match="traffic model not supported"):
        mk("bursty").arrival_kinds()
    with pytest.raises(AssertionError):
        mk("heterogeneous", []).arrival_kinds()
    # 1-D channel_switch broadcasts over agents (run_ippo_combinatorial.py:34)
    s = EnvSpec("comb", 3, 4, [2, 2, 2], [1] * 3, 5, None, None, 10, "aperiodic", [], False, np.array([.1, .2, .3, .4]))
    assert s.switch.shape == (3, 4) and np.all(s.switch[2] == [.1, .2, .3, .4])
    # chsel needs C+1 switch probabilities (channel_selection_env.py:105)
    with pytest.raises(IndexError):
        EnvSpec("chsel", 3, 4, [2, 2, 2], [1] * 3, 5, None, None, 10, "aperiodic", [], False, np.array([.1] * 4))


def test_mask_packing_roundtrip():
    from d2dhip.envbatch import pack_masks
    rng = np.random.default_rng(0)
    for C in (1, 5, 8, 12, 16, 23, 32):
        bits = rng.integers(0, 2, size=(7, 3, C))
        m = pack_masks(bits, C)
        raw = np.ascontiguousarray(m).view(np.uint8).reshape(7, 3, -1)
        back = np.unpackbits(raw, axis=2, bitorder="little")[:, :, :C]
        assert np.array_equal(back, bits)


def test_bernoulli_threshold_edges():
    from d2dhip.spec import bernoulli_threshold
    t = bernoulli_threshold([0.0, 1.0, 0.5, 0.2])
    assert list(t) == [0, 2 ** 32, 2 ** 31, int(np.floor(0.2 * 2 ** 32))]


def _apply_gather(codes, buffers, chan, ack):
    """Resolve d2d_env_single_gather_map codes against one env's buffers [N][D], chan [N], ack."""
    out = np.zeros(codes.shape[0], dtype=np.float64)
    for i, c in enumerate(codes):
        if c == -1:
            out[i] = ack
        elif c >= 0:
            j, q = c >> 6, c & 63
            out[i] = chan[j] if q == 32 else buffers[j, q]
    return out


def d2denv_fixtures():
    import glob
    from conftest import GOLDEN
    return sorted(glob.glob(os.path.join(GOLDEN, "d2denv_*.npz")))


@pytest.mark.parametrize("path", d2denv_fixtures(), ids=os.path.basename)
def test_single_gather_map_reproduces_reference_obs(path):
    """The host-built gather table (what the single_kernel's coalesced obs/state writes
    resolve through) rebuilds every recorded D2DEnv obs / state (env.py:91-98, 198-205)
    from the recorded buffers, channel states and ACKs."""
    import d2dhip
    from conftest import load_params
    from envs.env import D2DEnv
    lib = d2dhip.load()
    z = np.load(path)
    p = load_params(z)
    env = D2DEnv(**{k: v for k, v in p.items() if k != "verbose"})
    s = env.spec
    assert np.array_equal(s.obs_len, z["obs_dims"]) and s.S == int(z["state_dim"])
    assert [sp.shape[0] for sp in env.observation_space] == list(z["obs_dims"])     # env.py:43-45
    assert env.state_space.shape == (s.S,) and [a.n for a in env.action_space] == [2] * s.N
    codes = s.gather_map(lib)
    assert codes.shape == (s.N * s.F + s.S,)
    obs_codes, st_codes = codes[: s.N * s.F].reshape(s.N, s.F), codes[s.N * s.F:]
    for t in range(z["obs"].shape[0]):
        b, h, a = z["buffers"][t], z["chan"][t], float(z["ack"][t])
        for k in range(s.N):
            want = np.zeros(s.F, dtype=np.float32)
            want[: z["obs"].shape[2]] = z["obs"][t, k]
            assert np.array_equal(_apply_gather(obs_codes[k], b, h, a).astype(np.float32), want), (t, k)
        assert np.array_equal(_apply_gather(st_codes, b, h, a).astype(np.float32), z["state"][t]), t
    for w in range(z["reset_obs"].shape[0]):
        st = _apply_gather(st_codes, z["reset_buffers"][w], z["reset_chan"][w], 0.0)
        assert np.array_equal(st.astype(np.float32), z["reset_state"][w])


def test_single_gather_map_rejects_bad_neighbourhoods():
    import d2dhip
    lib = d2dhip.load()
    d = np.array([3, 3], dtype=np.int32)
    ptr = np.array([0, 1, 2], dtype=np.int32)
    idx = np.array([1, 5], dtype=np.int32)            # 5 is not an agent
    out = np.zeros(64, dtype=np.int32)
    rc = lib.d2d_env_single_gather_map(2, d.ctypes.data, ptr.ctypes.data, idx.ctypes.data, 5, out.ctypes.data, 64)
    assert rc == -1 and b"out of range" in lib.d2d_last_error()
    idx = np.array([1, 0], dtype=np.int32)
    rc = lib.d2d_env_single_gather_map(2, d.ctypes.data, ptr.ctypes.data, idx.ctypes.data, 4, out.ctypes.data, 64)
    assert rc == -1 and b"obs_dim" in lib.d2d_last_error()  # needs 3 + 1 + 1 = 5
    rc = lib.d2d_env_single_gather_map(2, d.ctypes.data, ptr.ctypes.data, idx.ctypes.data, 5, out.ctypes.data, 64)
    assert rc == 2 * 5 + 3 + 3 + 2 + 1
    from envs.env import D2DEnv
    with pytest.raises(ValueError, match="0 or 1"):
        D2DEnv(2, np.array([3, 3]), np.ones(2))._pack_actions([0, 2])
