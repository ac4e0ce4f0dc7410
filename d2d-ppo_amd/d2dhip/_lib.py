"""ctypes binding of libd2dhip.so (the C ABI declared in include/d2d_hip.h).

The library is built in-tree (`python __graft_entry__.py build` or
`make -C d2d-ppo_amd`) for gfx950 and loaded AFTER torch, so that it binds to
the HIP runtime torch already mapped (same SONAME libamdhip64.so.7): device
pointers and streams are then shared with torch.  There is no CPU fallback:
every entry point raises if the library cannot be loaded or no GPU is present.
"""
import ctypes
import os
import sys

import torch  # noqa: F401  (must be imported before the HIP library is loaded)

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_DIR, "lib", "libd2dhip.so")
# A/B timing builds only (tools/gpu/ablate_update.py): another in-tree build of the same library.
# Those builds drop parts of the update on purpose (wrong gradients), so the variable is honoured
# only together with an explicit D2D_ALLOW_ABLATION=1, loudly, and the learners refuse to train on it.
# "asan" is the host-sanitizer build (make -C d2d-ppo_amd asan, run only by tests/test_sanitizers_cpu.py
# on a GPU-less host): correct, but never a product library either.
VARIANT = os.environ.get("D2D_LIB_VARIANT") or None
if VARIANT:
    if VARIANT != "asan" and os.environ.get("D2D_ALLOW_ABLATION") != "1":
        raise RuntimeError(f"D2D_LIB_VARIANT={VARIANT} selects an ablation build of libd2dhip (wrong results "
                           f"by design); set D2D_ALLOW_ABLATION=1 as well to load it, or unset it")
    LIB_PATH = (os.path.join(PKG_DIR, "build", "asan", "libd2dhip_asan.so") if VARIANT == "asan"
                else os.path.join(PKG_DIR, "lib", f"libd2dhip_{VARIANT}.so"))
    print(f"[d2dhip] WARNING: loading {'sanitizer' if VARIANT == 'asan' else 'ablation'} build {LIB_PATH} "
          f"(not a product library)", file=sys.stderr, flush=True)


def refuse_ablation(what):
    """Product entry points (training, smoke) must not run on an ablation build."""
    if VARIANT:
        raise RuntimeError(f"{what} refuses the ablation build libd2dhip_{VARIANT}.so (D2D_LIB_VARIANT)")

D2D_ENV_COMBINATORIAL, D2D_ENV_CHANNEL_SELECTION, D2D_ENV_SINGLE = 0, 1, 2
D2D_ARRIVAL_POISSON, D2D_ARRIVAL_SCHEDULED_BERNOULLI, D2D_ARRIVAL_NONE = 0, 1, 2
ABI_VERSION = 15
D2D_OBS_F32, D2D_OBS_U8 = 0, 1
D2D_OPT_NT_STORES = 1
D2D_OPT_POLICY_F32_MFMA = 2
D2D_OPT_GRU_GRAD_HISTORY = 3  # 1: d2d_gru_grad through the global row history even where the LDS path applies
D2D_OPT_POLICY_CRITIC_SPLIT = 4  # 1: the iPPO critic value as its own launch beside the actor (bitwise the same)
D2D_OPT_CRITIC_GRAD_ROWS = 5  # 1: d2d_ppo_critic_grad on the sample-on-rows kernel of rounds 2-4 (A/B)
D2D_OPT_FUSED_SLICE = 6  # envs per workgroup of d2d_comb_policy_fused_step: 32 (0 = default) or 64

_p = ctypes.c_void_p


class EnvDesc(ctypes.Structure):
    _fields_ = [("env_kind", ctypes.c_int32), ("n_agents", ctypes.c_int32), ("n_channels", ctypes.c_int32),
                ("max_deadline", ctypes.c_int32), ("obs_dim", ctypes.c_int32), ("state_dim", ctypes.c_int32),
                ("state_stride", ctypes.c_int32), ("n_envs", ctypes.c_int32), ("env_base", ctypes.c_uint64),
                ("seed", ctypes.c_uint64), ("agents", _p), ("flip_thr", _p), ("arrival_kind_host", _p),
                ("period_host", _p), ("offset_host", _p), ("gather", _p), ("rng_offset", _p),
                ("poisson_cdf", _p)]


class EnvState(ctypes.Structure):
    _fields_ = [("buffers", _p), ("channels", _p), ("received", _p), ("discarded", _p), ("sel_quality", _p),
                ("sel_count", _p)]


class EnvOut(ctypes.Structure):
    _fields_ = [("obs", _p), ("state", _p), ("reward", _p), ("ack", _p), ("success", _p), ("obs_record", _p),
                ("state_bf16", _p), ("state_bf16_ld", ctypes.c_int64)]


def record_bytes(obs_dim):
    """D2D_RECORD_BYTES: row bytes of the compact obs record (32 per chunk of 32 network inputs)."""
    return 32 * ((int(obs_dim) + 32) // 32)


class EnvReplay(ctypes.Structure):
    _fields_ = [("flips", _p), ("arrivals", _p)]


class MlpDesc(ctypes.Structure):
    _fields_ = [("n_agents", ctypes.c_int32), ("n_envs", ctypes.c_int32), ("obs_dim", ctypes.c_int32),
                ("hidden", ctypes.c_int32), ("n_out", ctypes.c_int32), ("kind", ctypes.c_int32),
                ("w1", _p), ("b1", _p), ("w2", _p), ("b2", _p), ("v1", _p), ("c1", _p), ("v2", _p), ("c2", _p),
                ("seed", ctypes.c_uint64), ("env_base", ctypes.c_uint64), ("rng_offset", _p),
                ("obs_format", ctypes.c_int32), ("reserved", ctypes.c_int32), ("obs_signed", _p)]


class GruDesc(ctypes.Structure):
    _fields_ = [("n_agents", ctypes.c_int32), ("n_envs", ctypes.c_int32), ("obs_dim", ctypes.c_int32),
                ("hidden", ctypes.c_int32), ("n_out", ctypes.c_int32), ("kind", ctypes.c_int32),
                ("history_len", ctypes.c_int32), ("episode_length", ctypes.c_int32),
                ("w_ih", _p), ("w_hh", _p), ("b_ih", _p), ("b_hh", _p), ("w1", _p), ("b1", _p), ("w2", _p), ("b2", _p),
                ("seed", ctypes.c_uint64), ("env_base", ctypes.c_uint64), ("rng_offset", _p),
                ("obs_format", ctypes.c_int32), ("reserved", ctypes.c_int32), ("obs_signed", _p)]


# name -> (restype, argtypes)
_SIGS = {
    "d2d_env_reset": (ctypes.c_int, [ctypes.POINTER(EnvDesc), ctypes.POINTER(EnvState), ctypes.POINTER(EnvReplay),
                                      ctypes.POINTER(EnvOut), ctypes.c_uint32, _p]),
    "d2d_env_step": (ctypes.c_int, [ctypes.POINTER(EnvDesc), ctypes.POINTER(EnvState), _p, ctypes.POINTER(EnvReplay),
                                     ctypes.POINTER(EnvOut), ctypes.c_int32, ctypes.c_uint32, _p]),
    "d2d_sample_actions": (ctypes.c_int, [ctypes.POINTER(EnvDesc), _p, ctypes.c_uint64, ctypes.c_uint32, _p]),
    "d2d_mask_bytes": (ctypes.c_int, [ctypes.c_int32]),
    "d2d_env_single_gather_map": (ctypes.c_int, [ctypes.c_int32, _p, _p, _p, ctypes.c_int32, _p, ctypes.c_int64]),
    "d2d_buffer_words": (ctypes.c_int, [ctypes.c_int32]),
    "d2d_gae_scan": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _p, _p, _p, ctypes.c_double,
                                     ctypes.c_double, ctypes.c_int32, _p, _p, _p]),
    "d2d_gae_scan_tce": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _p, _p, _p,
                                         ctypes.c_double, ctypes.c_double, ctypes.c_int32, _p, _p, _p]),
    "d2d_colstats_tce": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _p, _p, _p, _p, _p]),
    "d2d_normalize_columns_tce": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _p, _p, _p, _p, _p]),
    "d2d_colstats_workspace": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32]),
    "d2d_colstats": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, _p, _p, _p, _p, _p]),
    "d2d_colstats_finalize": (ctypes.c_int, [ctypes.c_int32, _p, _p, ctypes.c_double, ctypes.c_int32, _p, _p, _p,
                                              _p]),
    "d2d_normalize_columns": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, _p, _p, _p, _p, _p]),
    "d2d_gae_moments_workspace": (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    "d2d_gae_scan_moments": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _p, _p, _p,
                                             ctypes.c_double, ctypes.c_double, ctypes.c_int32, ctypes.c_int32, _p, _p,
                                             _p, _p, ctypes.c_int64, _p]),
    "d2d_gae_scan_normalized": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _p, _p,
                                                _p, ctypes.c_double, ctypes.c_double, ctypes.c_int32, ctypes.c_int32,
                                                _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "d2d_normalize_pair": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _p, _p, _p,
                                           _p, _p, _p, _p, _p, _p]),
    "d2d_set_option": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32]),
    "d2d_happo_chain": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _p, _p, _p, _p, _p, _p]),
    "d2d_f32_to_bf16_exact": (ctypes.c_int, [ctypes.c_int64, _p, _p, _p, _p]),
    "d2d_states_to_bf16_exact": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, _p, _p,
                                                _p, _p]),
    "d2d_states_to_bf16_padded": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, _p, _p,
                                                  ctypes.c_int64, _p, _p]),
    "d2d_critic_dpre_blocks": (ctypes.c_int32, [ctypes.c_int64]),
    "d2d_critic_dpre_split": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int64, _p, _p, _p, _p, _p, ctypes.c_int32, _p]),
    "d2d_critic_dpre_split3": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int64, _p, _p, _p, _p, _p, ctypes.c_int32, _p]),
    "d2d_comb_policy_fused_step": (ctypes.c_int, [ctypes.POINTER(EnvDesc), ctypes.POINTER(EnvState), _p,
                                                   ctypes.POINTER(EnvOut), ctypes.c_int32, ctypes.c_uint32,
                                                   ctypes.POINTER(MlpDesc), ctypes.c_uint32, ctypes.c_int32, _p, _p, _p]),
    "d2d_policy_mlp_step": (ctypes.c_int, [ctypes.POINTER(MlpDesc), _p, _p, ctypes.c_uint32, ctypes.c_int32, _p, _p,
                                            _p, _p]),
    "d2d_ppo_workspace": (ctypes.c_int64, [ctypes.c_int32] * 6),
    "d2d_ppo_actor_grad": (ctypes.c_int, [ctypes.POINTER(MlpDesc), ctypes.c_int32, _p, _p, _p, _p, _p, _p,
                                           ctypes.c_float, ctypes.c_float, ctypes.c_float, _p, _p, _p, _p, _p, _p,
                                           ctypes.c_int64, _p]),
    "d2d_ppo_critic_grad": (ctypes.c_int, [ctypes.POINTER(MlpDesc), ctypes.c_int32, _p, _p, _p, ctypes.c_float,
                                            _p, _p, _p, _p, _p, _p, ctypes.c_int64, _p]),
    "d2d_ppo_critic_grad_values": (ctypes.c_int, [ctypes.POINTER(MlpDesc), ctypes.c_int32, _p, _p, _p, ctypes.c_float,
                                                   _p, _p, _p, _p, _p, _p, ctypes.c_int64, _p, _p, _p]),
    "d2d_central_critic_blocks": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int64]),
    "d2d_central_critic_image_bytes": (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32]),
    "d2d_central_critic_fwd": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64, _p, _p, _p,
                                               _p, _p, _p, _p, _p, _p, _p, ctypes.c_int32, _p]),
    "d2d_central_critic_dw1_workspace": (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64]),
    "d2d_central_critic_dw1": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64, _p, _p, _p,
                                               ctypes.c_int64, _p, _p]),
    "d2d_policy_gru": (ctypes.c_int, [ctypes.POINTER(GruDesc), ctypes.c_int32, _p, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_int32, _p, ctypes.c_uint32, ctypes.c_int32, _p, _p, _p]),
    "d2d_gru_carry_floats": (ctypes.c_int64, [ctypes.POINTER(GruDesc)]),
    "d2d_policy_gru_carry": (ctypes.c_int, [ctypes.POINTER(GruDesc), ctypes.c_int32, _p, ctypes.c_int32, _p,
                                             ctypes.c_uint32, ctypes.c_int32, _p, _p, _p, ctypes.c_int32, _p]),
    "d2d_gru_grad_workspace": (ctypes.c_int64, [ctypes.POINTER(GruDesc), ctypes.c_int32]),
    "d2d_gru_grad": (ctypes.c_int, [ctypes.POINTER(GruDesc), ctypes.c_int32, _p, _p, _p, _p, _p, _p, ctypes.c_float,
                                     ctypes.c_float, ctypes.c_float, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p,
                                     ctypes.c_int64, _p]),
    "d2d_last_error": (ctypes.c_char_p, []),
    "d2d_abi_version": (ctypes.c_int, []),
}

EXPORTED = tuple(_SIGS)

_lib = None


class D2DHipError(RuntimeError):
    pass


def _hip_runtimes_mapped():
    try:
        with open("/proc/self/maps") as fh:
            return sorted({ln.split()[-1] for ln in fh if "libamdhip64" in ln})
    except OSError:
        return []


def load(check_single_runtime=True):
    """Load libd2dhip.so (no GPU needed just to load and inspect the exports)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise D2DHipError(f"HIP extension not built: {LIB_PATH} is missing (run `python __graft_entry__.py build`)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    if lib.d2d_abi_version() != ABI_VERSION:
        raise D2DHipError(f"libd2dhip ABI {lib.d2d_abi_version()} != {ABI_VERSION}")
    if check_single_runtime:
        rts = _hip_runtimes_mapped()
        if len(rts) > 1:
            raise D2DHipError(f"two HIP runtimes mapped in this process: {rts}")
    _lib = lib
    return lib


def require_gpu():
    if not torch.cuda.is_available():
        raise D2DHipError("the D2D-PPO HIP path needs a ROCm GPU (torch.cuda.is_available() is False); "
                          "there is no CPU fallback")
    return load()


def check(rc, what):
    if rc != 0:
        msg = _lib.d2d_last_error().decode() if _lib is not None else ""
        if rc == -1:
            raise ValueError(f"{what}: {msg}")
        if rc == -2:
            raise NotImplementedError(f"{what}: {msg}")
        raise D2DHipError(f"{what} failed ({rc}): {msg}")


def ptr(t):
    """Raw device pointer of a torch tensor (or None)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)
