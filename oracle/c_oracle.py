"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the C oracle (oracle/c/d2d_oracle.c).

Used by tests/ (bit-exact checks of the HIP kernels' Philox mode at sizes the
numpy oracle is too slow for) and by bench.py's cpu_baseline leg.  Never by
the product path.
"""
import ctypes
import os

import numpy as np

from . import philox
from .env_oracle import _Spec

HERE = os.path.dirname(os.path.abspath(__file__))
# D2D_ORACLE_ASAN=1: the AddressSanitizer / UBSan build (make -C oracle asan; tests/test_sanitizers_cpu.py)
LIB_PATH = os.path.join(HERE, "build", "asan/libd2d_oracle_asan.so" if os.environ.get("D2D_ORACLE_ASAN") == "1"
                        else "libd2d_oracle.so")

_p = ctypes.c_void_p


class OSpec(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("N", ctypes.c_int), ("C", ctypes.c_int), ("D", ctypes.c_int),
                ("F", ctypes.c_int), ("S", ctypes.c_int),
                ("d", _p), ("w", _p), ("state_off", _p), ("arr_kind", _p),
                ("lam", _p), ("p0", _p), ("period", _p), ("offset", _p),
                ("q_thr", _p), ("flip_thr", _p), ("seed", ctypes.c_uint64), ("env_base", ctypes.c_uint64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"C oracle not built: run `make -C {HERE}`")
        _lib = ctypes.CDLL(LIB_PATH)
        for fn in ("oracle_reset", "oracle_step", "oracle_sample_actions", "oracle_max_threads"):
            getattr(_lib, fn).restype = ctypes.c_int
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class COracle:
    """Batched C oracle over E envs.  Arrays are numpy (unpacked layout)."""

    def __init__(self, kind, params, n_envs, seed=0, env_base=0, nthreads=0):
        s = _Spec(kind, **params)
        self.spec, self.kind, self.E, self.nthreads = s, kind, int(n_envs), int(nthreads)
        N, C, D = s.N, s.C, s.D
        arr_kind = np.full(N, 2, dtype=np.int32)
        tm = s.traffic_model
        if tm == "aperiodic":
            arr_kind[:] = 0
        elif tm == "periodic":
            arr_kind[:] = 1
        elif tm == "heterogeneous":
            arr_kind[s.aperiodic_devices] = 0
            arr_kind[s.periodic_devices] = 1
        self._keep = dict(
            d=s.d.astype(np.int32), w=s.w.astype(np.int32), state_off=s.state_off.astype(np.int32),
            arr_kind=arr_kind, lam=s.lam.astype(np.float64), p0=np.exp(-s.lam.astype(np.float64)),
            period=s.period.astype(np.float64), offset=s.offsets.astype(np.float64),
            q_thr=philox.threshold(s.q), flip_thr=philox.threshold(s.switch.reshape(-1)[: (N * C if kind == "comb" else C + 1)]))
        k = self._keep
        self.ospec = OSpec(0 if kind == "comb" else 1, N, C, D, s.F, s.S, *(_ptr(k[n]) for n in (
            "d", "w", "state_off", "arr_kind", "lam", "p0", "period", "offset", "q_thr", "flip_thr")),
            int(seed), int(env_base))
        E = self.E
        self.buf = np.zeros((E, N, D), dtype=np.uint8)
        self.chan = np.ones((E, N, C) if kind == "comb" else (E, C + 1), dtype=np.uint8)
        self.recv = np.zeros((E, N), dtype=np.uint32)
        self.disc = np.zeros((E, N), dtype=np.uint32)
        self.selq = np.zeros(E, dtype=np.uint32)
        self.seln = np.zeros(E, dtype=np.uint32)
        self.timestep = 0

    def reset(self, rng_step=0, arrivals=None, want_obs=True, want_state=True):
        s = self.spec
        obs = np.zeros((self.E, s.N, s.F), dtype=np.float32) if want_obs else None
        state = np.zeros((self.E, s.S), dtype=np.float32) if want_state else None
        arr = None if arrivals is None else np.ascontiguousarray(arrivals, dtype=np.uint8)
        lib().oracle_reset(ctypes.byref(self.ospec), self.E, ctypes.c_uint32(rng_step), _ptr(arr), _ptr(self.buf),
                           _ptr(self.chan), _ptr(self.recv), _ptr(self.disc), _ptr(self.selq), _ptr(self.seln),
                           _ptr(obs), _ptr(state), self.nthreads)
        self.timestep = 0
        return dict(obs=obs, state=state)

    def step(self, actions, rng_step, flips=None, arrivals=None, want_obs=True, want_state=True):
        s = self.spec
        self.timestep += 1
        obs = np.zeros((self.E, s.N, s.F), dtype=np.float32) if want_obs else None
        state = np.zeros((self.E, s.S), dtype=np.float32) if want_state else None
        reward = np.zeros(self.E, dtype=np.int32)
        ack = np.zeros((self.E, s.C if self.kind == "comb" else s.C + 1), dtype=np.float64)
        success = np.zeros((self.E, s.N), dtype=np.uint8)
        act = np.ascontiguousarray(actions, dtype=np.uint8)
        fl = None if flips is None else np.ascontiguousarray(flips, dtype=np.uint8)
        arr = None if arrivals is None else np.ascontiguousarray(arrivals, dtype=np.uint8)
        rc = lib().oracle_step(ctypes.byref(self.ospec), self.E, self.timestep, ctypes.c_uint32(rng_step), _ptr(act),
                               _ptr(fl), _ptr(arr), _ptr(self.buf), _ptr(self.chan), _ptr(self.recv), _ptr(self.disc),
                               _ptr(self.selq), _ptr(self.seln), _ptr(obs), _ptr(state), _ptr(reward), _ptr(ack),
                               _ptr(success), self.nthreads)
        if rc != 0:
            raise ValueError("oracle_step: unsupported shape")
        return dict(obs=obs, state=state, reward=reward, ack=ack, success=success,
                    done=self.timestep >= s.episode_length)

    def sample_actions(self, rng_step, p=0.1):
        s = self.spec
        shape = (self.E, s.N, s.C) if self.kind == "comb" else (self.E, s.N)
        out = np.zeros(shape, dtype=np.uint8)
        thr = int(philox.threshold(p))
        lib().oracle_sample_actions(ctypes.byref(self.ospec), self.E, ctypes.c_uint32(rng_step), ctypes.c_uint64(thr),
                                    _ptr(out), self.nthreads)
        return out
