"""The compact obs record (C ABI D2D_OBS_U8, include/d2d_hip.h d2d_env_out.obs_record).

The combinatorial env's observation (combinatorial_env.py:199-206) is made of packet counts (uint8
buffer cells), channel bits and ACKs in {-1, 0, 1}: every value is an integer that fits one byte.  So is the
D2DEnv's (envs/env.py:89-95: the neighbours' buffers and channel bits, the last feedback in {-1, 0, 1}; ABI 14).
The env kernel can write each obs row as bytes, padded to 32 per chunk of 32 network inputs, and
the policy / update / GRU kernels read it instead of the fp32 rows: 32 bytes per (env, agent) slot
instead of 4 * obs_dim (120 at the c3 headline config).  The decoded values are the same floats,
so every result is bit-identical to the fp32 path.

ObsRecord pairs the byte tensor [..., N, R] with the per-agent int8-column masks [N][R / 32]
(bit b of word c: column 32c + b is signed) the kernels take as `obs_signed`.
"""
import numpy as np
import torch

from . import _lib


def signed_masks(spec, gather=None):
    """uint32 [N][R / 32] int8-column masks of an EnvSpec's record: combinatorial env, agent k's ACK columns
    [w_k + C, w_k + 2C) (obs layout of combinatorial_env.py:199-206); D2DEnv (kind 'single', ABI 14), the column
    of the agent's last feedback (env.py:94; gather code -1 of d2d_env_single_gather_map, `gather` = the host codes)."""
    if spec.kind == "single":
        if gather is None:
            raise ValueError("the D2DEnv record's masks need the env's gather codes")
        R = _lib.record_bytes(spec.F)
        codes = np.asarray(gather)[: spec.N * spec.F].reshape(spec.N, spec.F)
        m = np.zeros((spec.N, R // 32), dtype=np.uint64)
        for k, col in zip(*np.nonzero(codes == -1)):
            m[k, col // 32] |= np.uint64(1) << np.uint64(col % 32)
        return m.astype(np.uint32)
    if spec.kind != "comb":
        raise NotImplementedError("the compact obs record exists for the combinatorial env and the D2DEnv only")
    R = _lib.record_bytes(spec.F)
    m = np.zeros((spec.N, R // 32), dtype=np.uint64)
    for k in range(spec.N):
        w = int(spec.w[k])
        for col in range(w + spec.C, w + 2 * spec.C):
            m[k, col // 32] |= np.uint64(1) << np.uint64(col % 32)
    return m.astype(np.uint32)


class ObsRecord:
    """data: uint8 [..., N, R] (contiguous, 16-byte aligned); obs_dim: F; signed: int32 [N][R / 32] device
    tensor (the uint32 masks).  `shape` is the logical obs shape [..., N, F]."""

    def __init__(self, data, obs_dim, signed):
        if data.dtype != torch.uint8:
            raise ValueError("record data must be uint8")
        R = _lib.record_bytes(obs_dim)
        if data.shape[-1] != R:
            raise ValueError(f"record rows of {data.shape[-1]} bytes, expected {R} for obs_dim {obs_dim}")
        if signed.dtype != torch.int32 or tuple(signed.shape) != (data.shape[-2], R // 32):
            raise ValueError(f"signed masks must be int32 [{data.shape[-2]}][{R // 32}]")
        self.data, self.obs_dim, self.signed = data, int(obs_dim), signed
        self._host = None

    def signed_host(self):
        """int32 numpy copy of the masks (read once, then cached; slices share the tensor)."""
        if self._host is None:
            self._host = self.signed.cpu().numpy()
        return self._host

    @classmethod
    def empty(cls, lead, spec, signed, device):
        R = _lib.record_bytes(spec.F)
        return cls(torch.zeros(tuple(lead) + (spec.N, R), dtype=torch.uint8, device=device), spec.F, signed)

    @property
    def shape(self):
        return tuple(self.data.shape[:-1]) + (self.obs_dim,)

    @property
    def device(self):
        return self.data.device

    def is_contiguous(self):
        return self.data.is_contiguous()

    def __getitem__(self, idx):
        """Slices of the leading (slot / env) dims."""
        r = ObsRecord(self.data[idx], self.obs_dim, self.signed)
        r._host = self._host
        return r

    def data_ptr(self):
        return self.data.data_ptr()

    def decode(self):
        """float32 [..., N, F]: the fp32 obs the record encodes (host-side views, tests)."""
        d = self.data[..., : self.obs_dim]
        sg = self.signed.to(torch.int64) & 0xFFFFFFFF
        cols = torch.arange(self.obs_dim, device=d.device)
        neg = ((sg[:, cols // 32] >> (cols % 32)) & 1).bool()       # [N][F]
        u = d.to(torch.float32)
        s = d.view(torch.int8).to(torch.float32)
        return torch.where(neg, s, u)


def obs_arg(obs):
    """(device pointer, obs_format, obs_signed pointer) of an fp32 obs tensor or an ObsRecord."""
    if isinstance(obs, ObsRecord):
        if not obs.data.is_contiguous() or obs.data.data_ptr() % 16:
            raise ValueError("the obs record must be contiguous and 16-byte aligned")
        return obs.data.data_ptr(), _lib.D2D_OBS_U8, obs.signed.data_ptr()
    if obs.dtype != torch.float32 or not obs.is_contiguous():
        raise ValueError("obs must be a contiguous float32 tensor (or an ObsRecord)")
    return obs.data_ptr(), _lib.D2D_OBS_F32, None


def set_format(desc, obs):
    """Fill a MlpDesc / GruDesc's obs_format / obs_signed for `obs`; returns the obs pointer."""
    p, fmt, sg = obs_arg(obs)
    desc.obs_format = fmt
    desc.obs_signed = sg
    return p
