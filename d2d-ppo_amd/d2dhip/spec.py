"""Derive the per-agent device tables from the reference constructor kwargs.

Mirrors how the reference envs interpret their arguments:
  traffic models     envs/combinatorial_env.py:66-85 (reset), 178-196 (step)
                     envs/channel_selection_env.py:54-73, 159-177
  spaces             envs/combinatorial_env.py:47-58, channel_selection_env.py:41-46
  channel_switch     combinatorial_env.py:42-45 (default zeros((N, C)); a 1-D
                     vector broadcasts over agents), channel_selection_env.py:35-38
                     (C+1 scalar probabilities, channel 0 included),
                     envs/env.py:33-37, 105-107 (one flip probability per agent, default 0.2)
  neighbourhoods     envs/env.py:39-49 (obs of agent k = buffers + channel states of
                     nbr(k), in list order, + the ack; default nbr(k) = [k])
"""
import numpy as np

COMB, CHSEL, SINGLE = "comb", "chsel", "single"

AGENT_DTYPE = np.dtype([("deadline", "u1"), ("obs_width", "u1"), ("arrival_kind", "u1"), ("reserved", "u1"),
                        ("state_offset", "<i4"), ("lam", "<f8"), ("pois_p0", "<f8"), ("arrival_thr", "<u8")])
assert AGENT_DTYPE.itemsize == 32

POISSON, SCHEDULED, NONE = 0, 1, 2


def bernoulli_threshold(p):
    """Bernoulli(p) drawn from one uint32 word r as r < floor(p * 2**32)."""
    p = np.clip(np.asarray(p, dtype=np.float64), 0.0, 1.0)
    return np.floor(p * 4294967296.0).astype(np.uint64)


POISSON_TABLE = 256


def poisson_cdf_table(lam, kinds):
    """Inverse-CDF thresholds of the Philox-mode Poisson arrival draw, uint32 [N][256].

    The draw is the sequential inversion "x = 0; p = F = exp(-lam); while u >= F and x < 255:
    x += 1; p = p * lam / x; F += p" of u = r * 2^-32 (d2d_hip.h, oracle/philox.py
    poisson_inversion).  For an integer word r, u >= F_x  <=>  r >= ceil(F_x * 2^32), so with
    t[x] = min(ceil(F_x * 2^32), 2^32) - 1 the result is the number of leading entries with
    r > t[x]: the F_x are accumulated here in the same IEEE double operations, the table is
    nondecreasing, and t[255] = 2^32 - 1 stops every search at the cap.  Rows of agents that do
    not draw Poisson arrivals are all 2^32 - 1 (never read).
    """
    lam = np.asarray(lam, dtype=np.float64)
    N = lam.shape[0]
    t = np.full((N, POISSON_TABLE), 0xFFFFFFFF, dtype=np.uint64)
    pois = np.asarray(kinds) == POISSON
    if pois.any():
        lp = lam[pois]
        # a threshold ceil(F_x * 2^32) - 1 needs F_x > 0: exp(-lam) underflows near lam = 745, and the
        # uint8 cells already cap the mean at 64 (EnvSpec.agent_table), so refuse such means here too
        if np.any(~(lp <= 64.0)):
            raise NotImplementedError("Poisson means > 64 overflow the uint8 buffer cells")
        p = np.exp(-lam)[pois]  # the agent table's pois_p0, computed over the same array
        F = p.copy()
        cols = [F.copy()]
        for x in range(1, POISSON_TABLE - 1):
            p = (p * lp) / float(x)
            F = F + p
            cols.append(F.copy())
        Fx = np.stack(cols, axis=1)                                   # [n][255]: F_0 .. F_254
        ce = np.minimum(np.ceil(Fx * 4294967296.0), 4294967296.0)     # exact: power-of-two scaling
        t[pois, :POISSON_TABLE - 1] = ce.astype(np.uint64) - np.uint64(1)
    return t.astype(np.uint32)


def buffer_words(D):
    return 1 if D <= 4 else 2 if D <= 8 else 3 if D <= 12 else 4 if D <= 16 else 8


def mask_bytes(C):
    return 1 if C <= 8 else 2 if C <= 16 else 4


class EnvSpec:
    def __init__(self, kind, n_agents, n_channels, deadlines, lbdas, period, arrival_probs, offsets, episode_length,
                 traffic_model, periodic_devices, homogeneous_size, channel_switch, neighbourhoods=None):
        self.kind = kind
        N, C = int(n_agents), int(n_channels)
        self.N, self.C = N, C
        d = np.asarray(deadlines).astype(np.int64).reshape(-1)
        if d.shape[0] != N:
            raise ValueError(f"deadlines has {d.shape[0]} entries for {N} agents")
        if d.min() < 1:
            raise ValueError("deadlines must be >= 1")
        self.d = d
        self.D = int(d.max())
        self.homog = bool(homogeneous_size) and kind == COMB
        self.w = np.full(N, self.D) if self.homog else d.copy()
        self.episode_length = episode_length
        self.traffic_model = traffic_model
        pdev = [] if periodic_devices is None else [int(i) for i in np.asarray(periodic_devices).reshape(-1)]
        self.periodic_devices = pdev
        self.aperiodic_devices = [i for i in range(N) if i not in pdev]

        def per_agent(x, default):
            if x is None:
                return np.full(N, default, dtype=np.float64)
            a = np.asarray(x, dtype=np.float64)
            return np.full(N, float(a)) if a.ndim == 0 else np.broadcast_to(a.reshape(-1), (N,)).copy()

        self.lam = per_agent(lbdas, 0.0)
        self.q = per_agent(arrival_probs, 0.0)
        self.period = per_agent(period, 1.0)
        self.offsets = per_agent(offsets, 0.0)
        if kind == COMB:
            cs = np.zeros((N, C)) if channel_switch is None else np.broadcast_to(
                np.asarray(channel_switch, dtype=np.float64), (N, C))
            self.switch = np.array(cs, dtype=np.float64)
            self.F = self.D + 2 * C
            self.S = int(d.sum()) + C * (N + 1)
        elif kind == SINGLE:
            if C != 1:
                raise ValueError("the D2DEnv has exactly one channel")
            cs = 0.2 if channel_switch is None else channel_switch
            self.switch = np.broadcast_to(np.asarray(cs, dtype=np.float64), (N,)).copy()
            nbr = [[k] for k in range(N)] if neighbourhoods is None else \
                [[int(j) for j in np.asarray(nb).reshape(-1)] for nb in neighbourhoods]
            if len(nbr) != N:
                raise ValueError(f"neighbourhoods has {len(nbr)} entries for {N} agents")
            for nb in nbr:
                if any(j < 0 or j >= N for j in nb):
                    raise IndexError(f"neighbour index out of range in {nb}")
            self.nbr = nbr
            self.nbr_ptr = np.concatenate([[0], np.cumsum([len(nb) for nb in nbr])]).astype(np.int32)
            self.nbr_idx = np.array([j for nb in nbr for j in nb], dtype=np.int32)
            self.F = int(max(int(d[nb].sum()) + len(nb) + 1 for nb in nbr))
            self.S = int(d.sum()) + N + 1
        else:
            cs = np.zeros(N) if channel_switch is None else np.asarray(channel_switch, dtype=np.float64).reshape(-1)
            if cs.shape[0] < C + 1:
                # the reference indexes channel_switch[k] for k in range(C+1) (channel_selection_env.py:105)
                raise IndexError(f"channel_switch needs at least n_channels+1={C + 1} entries, got {cs.shape[0]}")
            self.switch = cs[: C + 1].copy()
            self.F = self.D + C + 1
            self.S = int(d.sum()) + C + 1
        self.state_stride = (self.S + 3) // 4 * 4
        self.state_off = np.concatenate([[0], np.cumsum(d)[:-1]]).astype(np.int64)
        if kind == COMB:
            self.obs_len = self.w + 2 * C
        elif kind == SINGLE:
            self.obs_len = np.array([int(d[nb].sum()) + len(nb) + 1 for nb in self.nbr], dtype=np.int64)
        else:
            self.obs_len = d + C + 1
        self.DW = buffer_words(self.D)
        self.mask_bytes = mask_bytes(C) if kind == COMB else 4
        if self.D > 32 or self.D > 255:
            raise NotImplementedError("max deadline > 32 is not supported by the HIP kernels")
        if N > 1024:
            raise NotImplementedError("n_agents > 1024 is not supported by the HIP kernels")
        if kind == SINGLE and self.F > 1 << 24:
            raise NotImplementedError("neighbourhood observations longer than 2^24 floats")
        if (kind == COMB and C > 32) or (kind == CHSEL and C > 31):
            raise NotImplementedError("too many channels for the HIP kernels")

    def arrival_kinds(self):
        """Per-agent draw kind; raises like the reference's reset (ValueError /
        AssertionError) for an unknown model or an empty heterogeneous split."""
        N = self.N
        kinds = np.full(N, NONE, dtype=np.uint8)
        tm = self.traffic_model
        if tm == "aperiodic":
            kinds[:] = POISSON
        elif tm == "periodic":
            kinds[:] = SCHEDULED
        elif tm == "heterogeneous":
            assert len(self.periodic_devices) > 0 and len(self.aperiodic_devices) > 0, \
                "periodic_devices and aperiodic_devices must be non empty"
            kinds[self.aperiodic_devices] = POISSON
            kinds[self.periodic_devices] = SCHEDULED
        else:
            raise ValueError('traffic model not supported')
        if np.any(self.lam[kinds == POISSON] > 64):
            raise NotImplementedError("Poisson means > 64 overflow the uint8 buffer cells")
        return kinds

    def agent_table(self, kinds):
        t = np.zeros(self.N, dtype=AGENT_DTYPE)
        t["deadline"] = self.d
        t["obs_width"] = self.w
        t["arrival_kind"] = kinds
        t["state_offset"] = self.state_off
        t["lam"] = self.lam
        t["pois_p0"] = np.exp(-self.lam)
        t["arrival_thr"] = bernoulli_threshold(self.q)
        return t

    def poisson_table(self, kinds):
        return poisson_cdf_table(self.lam, kinds)

    def gather_map(self, lib):
        """D2DEnv obs/state gather codes (d2d_env_single_gather_map, host-only)."""
        import ctypes
        n = self.N * self.F + self.S
        out = np.zeros(n, dtype=np.int32)
        dl = np.ascontiguousarray(self.d, dtype=np.int32)
        rc = lib.d2d_env_single_gather_map(self.N, dl.ctypes.data, self.nbr_ptr.ctypes.data, self.nbr_idx.ctypes.data,
                                           self.F, out.ctypes.data, ctypes.c_int64(n))
        if rc != n:
            raise ValueError(f"d2d_env_single_gather_map: {lib.d2d_last_error().decode()}")
        return out

    def flip_thresholds(self):
        return bernoulli_threshold(self.switch.reshape(-1))
