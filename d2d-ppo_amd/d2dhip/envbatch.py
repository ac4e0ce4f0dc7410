"""Device-resident batch of E environments driven through the C ABI.

All state lives in HBM (torch tensors used as plain allocations); reset/step
are single kernel launches on the current torch stream, with no host
synchronisation — the learners and the benchmark chain them freely and the
whole rollout can be captured in a HIP graph.
"""
import numpy as np
import torch

from . import _lib
from .record import ObsRecord, signed_masks
from .spec import COMB, SINGLE, EnvSpec

_KIND_ID = {COMB: _lib.D2D_ENV_COMBINATORIAL, "chsel": _lib.D2D_ENV_CHANNEL_SELECTION, SINGLE: _lib.D2D_ENV_SINGLE}

_MASK_DTYPE = {1: torch.uint8, 2: torch.int16, 4: torch.int32}


class EnvBatch:
    def __init__(self, spec: EnvSpec, n_envs, device=None, seed=0, env_base=0):
        self.lib = _lib.require_gpu()
        self.spec = spec
        self.E = int(n_envs)
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise _lib.D2DHipError(f"EnvBatch needs a GPU device, got {self.device}")
        s, E, dev = spec, self.E, self.device
        self.kinds = spec.arrival_kinds()
        # per-agent tables (device) + arrival schedule (host)
        tab = spec.agent_table(self.kinds)
        self.agents = torch.from_numpy(tab.view(np.uint8).copy()).to(dev)
        self.flip_thr = torch.from_numpy(spec.flip_thresholds().view(np.int64).copy()).to(dev)
        self.poisson_cdf = torch.from_numpy(spec.poisson_table(self.kinds).view(np.int32).copy()).to(dev)
        self._kinds_host = np.ascontiguousarray(self.kinds, dtype=np.uint8)
        self._period_host = np.ascontiguousarray(spec.period, dtype=np.float64)
        self._offset_host = np.ascontiguousarray(spec.offsets, dtype=np.float64)
        # env state
        self.buffers = torch.zeros((E, s.N, s.DW), dtype=torch.int32, device=dev)
        if s.kind == COMB:
            self.channels = torch.zeros((E, s.N), dtype=_MASK_DTYPE[s.mask_bytes], device=dev)
            self.sel_quality = self.sel_count = None
        elif s.kind == SINGLE:
            # per-agent channel bit; sel_quality / sel_count hold channel_errors / n_collisions
            self.channels = torch.zeros((E, s.N), dtype=torch.uint8, device=dev)
            self.sel_quality = torch.zeros((E,), dtype=torch.int32, device=dev)
            self.sel_count = torch.zeros((E,), dtype=torch.int32, device=dev)
        else:
            self.channels = torch.zeros((E,), dtype=torch.int32, device=dev)
            self.sel_quality = torch.zeros((E,), dtype=torch.int32, device=dev)
            self.sel_count = torch.zeros((E,), dtype=torch.int32, device=dev)
        self.received = torch.zeros((E, s.N), dtype=torch.int32, device=dev)
        self.discarded = torch.zeros((E, s.N), dtype=torch.int32, device=dev)
        # persistent outputs (overwritten by every call unless `out_*` is given)
        self.obs = torch.zeros((E, s.N, s.F), dtype=torch.float32, device=dev)
        self.reward = torch.zeros((E,), dtype=torch.int32, device=dev)
        self._state = None
        self._ack = None
        self._success = None
        self._record = None
        # int8-column masks of the compact obs record (combinatorial env; D2DEnv from its gather codes)
        gather_host = spec.gather_map(self.lib) if s.kind == SINGLE else None
        self._signed_host = (signed_masks(s, gather_host).view(np.int32) if s.kind in (COMB, SINGLE) else None)
        self.signed = torch.from_numpy(self._signed_host).to(dev) if self._signed_host is not None else None
        self.gather = torch.from_numpy(gather_host).to(dev) if s.kind == SINGLE else None
        # device word added to rng_step by every kernel of this batch (and by the learner's policy
        # kernel): 0 for eager calls, set before replaying a captured rollout graph
        self.rng_off = torch.zeros(1, dtype=torch.int32, device=dev)
        self.desc = _lib.EnvDesc(
            _KIND_ID[s.kind], s.N, s.C, s.D, s.F, s.S, s.state_stride, E, int(env_base),
            int(seed) & 0xFFFFFFFFFFFFFFFF, self.agents.data_ptr(), self.flip_thr.data_ptr(),
            self._kinds_host.ctypes.data, self._period_host.ctypes.data, self._offset_host.ctypes.data,
            None if self.gather is None else self.gather.data_ptr(), self.rng_off.data_ptr(),
            self.poisson_cdf.data_ptr())
        self.st = _lib.EnvState(self.buffers.data_ptr(), self.channels.data_ptr(), self.received.data_ptr(),
                                self.discarded.data_ptr(),
                                None if self.sel_quality is None else self.sel_quality.data_ptr(),
                                None if self.sel_count is None else self.sel_count.data_ptr())
        self.rng_step = 0
        self.timestep = 0

    # ------------------------------------------------------------ buffers
    @property
    def state(self):
        if self._state is None:
            self._state = torch.zeros((self.E, self.spec.state_stride), dtype=torch.float32, device=self.device)
        return self._state

    @property
    def ack(self):
        if self._ack is None:
            s = self.spec
            if s.kind == COMB:
                self._ack = torch.zeros((self.E, s.C), dtype=torch.int8, device=self.device)
            elif s.kind == SINGLE:
                self._ack = torch.zeros((self.E,), dtype=torch.int8, device=self.device)
            else:
                self._ack = torch.zeros((self.E, s.C + 1), dtype=torch.float64, device=self.device)
        return self._ack

    @property
    def record(self):
        """Persistent compact obs record [E][N][R] (ObsRecord; combinatorial env and D2DEnv)."""
        if self._record is None:
            self._record = self.record_buffer(())
        return self._record

    def record_buffer(self, lead):
        """A zeroed ObsRecord [*lead][E][N][R] for rollout buffers (slice [t] per step)."""
        if self.signed is None:
            raise NotImplementedError("the compact obs record exists for the combinatorial env and the D2DEnv only")
        r = ObsRecord.empty(tuple(lead) + (self.E,), self.spec, self.signed, self.device)
        r._host = self._signed_host
        return r

    @property
    def success(self):
        if self._success is None:
            self._success = torch.zeros((self.E, self.spec.N), dtype=torch.uint8, device=self.device)
        return self._success

    def action_buffer(self):
        s = self.spec
        if s.kind == COMB:
            return torch.zeros((self.E, s.N), dtype=_MASK_DTYPE[s.mask_bytes], device=self.device)
        return torch.zeros((self.E, s.N), dtype=torch.uint8, device=self.device)

    # ------------------------------------------------------------- checks
    def _check_out(self, t, shape, dtype, name):
        if t is None:
            return
        if tuple(t.shape) != tuple(shape) or t.dtype != dtype or not t.is_contiguous() or t.device != self.device:
            raise ValueError(f"{name}: expected contiguous {dtype} {tuple(shape)} on {self.device}, got "
                             f"{t.dtype} {tuple(t.shape)} on {t.device}")

    def _replay(self, replay):
        if replay is None:
            return None, ()
        flips, arrivals = replay
        s = self.spec
        keep = []
        fp = ap = None
        if flips is not None:
            want = (self.E, s.N) if s.kind in (COMB, SINGLE) else (self.E,)
            dt = _MASK_DTYPE[s.mask_bytes] if s.kind == COMB else torch.uint8 if s.kind == SINGLE else torch.int32
            self._check_out(flips, want, dt, "replay flips")
            fp = flips.data_ptr()
            keep.append(flips)
        if arrivals is not None:
            self._check_out(arrivals, (self.E, s.N), torch.uint8, "replay arrivals")
            ap = arrivals.data_ptr()
            keep.append(arrivals)
        return _lib.EnvReplay(fp, ap), keep

    def _out(self, want_obs, want_state, want_ack, want_success, out_obs, out_state, out_reward, out_record=None,
             out_state_bf16=None):
        s = self.spec
        if isinstance(out_obs, ObsRecord):
            out_obs, out_record = None, out_obs
        rec = None
        if out_record is not None:
            if out_record.signed is not self.signed and not np.array_equal(out_record.signed_host(), self._signed_host):
                raise ValueError("out_record carries another env's signed-column masks")
            self._check_out(out_record.data, (self.E, s.N, _lib.record_bytes(s.F)), torch.uint8, "out_record")
            rec = out_record.data
            want_obs = False
        obs = out_obs if out_obs is not None else (self.obs if want_obs else None)
        state = out_state if out_state is not None else (self.state if want_state else None)
        reward = out_reward if out_reward is not None else self.reward
        self._check_out(obs, (self.E, s.N, s.F), torch.float32, "obs")
        self._check_out(state, (self.E, s.state_stride), torch.float32, "state")
        self._check_out(reward, (self.E,), torch.int32, "reward")
        ack = self.ack if want_ack else None
        succ = self.success if want_success else None
        o = _lib.EnvOut(*(None if t is None else t.data_ptr() for t in (obs, state, reward, ack, succ, rec)))
        if out_state_bf16 is not None:
            # [E][ld] bf16 rows with any row stride (a slot's rows of an env-major [E][T][ld] buffer): d2d_env_out.state_bf16
            x = out_state_bf16
            ld8 = -(-s.S // 8) * 8
            if (x.dtype != torch.bfloat16 or x.dim() != 2 or x.shape[0] != self.E or x.shape[1] < ld8 or x.stride(1) != 1
                    or x.device != self.device):
                raise ValueError(f"out_state_bf16: expected bf16 ({self.E}, >= {ld8}) rows on {self.device}, got "
                                 f"{x.dtype} {tuple(x.shape)} strides {x.stride()}")
            o.state_bf16, o.state_bf16_ld = x.data_ptr(), x.stride(0)
        return o, dict(obs=obs if rec is None else out_record, state=state, reward=reward, ack=ack, success=succ)

    # ---------------------------------------------------------- reset/step
    def reset(self, want_obs=True, want_state=False, replay_arrivals=None, out_obs=None, out_state=None,
              stream=None, out_state_bf16=None):
        o, res = self._out(want_obs, want_state, False, False, out_obs, out_state, None, out_state_bf16=out_state_bf16)
        rp, _keep = self._replay(None if replay_arrivals is None else (None, replay_arrivals))
        rc = self.lib.d2d_env_reset(self.desc, self.st, rp, o, self.rng_step, _lib.stream_ptr(stream))
        _lib.check(rc, "d2d_env_reset")
        self.rng_step += 1
        self.timestep = 0
        res.pop("reward")
        return res

    def step(self, actions, want_obs=True, want_state=False, want_ack=False, want_success=False, replay=None,
             out_obs=None, out_state=None, out_reward=None, stream=None, out_state_bf16=None):
        s = self.spec
        want_act = (self.E, s.N)
        dt = _MASK_DTYPE[s.mask_bytes] if s.kind == COMB else torch.uint8
        self._check_out(actions, want_act, dt, "actions")
        o, res = self._out(want_obs, want_state, want_ack, want_success, out_obs, out_state, out_reward,
                           out_state_bf16=out_state_bf16)
        rp, _keep = self._replay(replay)
        self.timestep += 1
        rc = self.lib.d2d_env_step(self.desc, self.st, actions.data_ptr(), rp, o, self.timestep, self.rng_step,
                                   _lib.stream_ptr(stream))
        _lib.check(rc, "d2d_env_step")
        self.rng_step += 1
        res["done"] = self.timestep >= s.episode_length
        return res

    def step_policy_fused(self, actions, out_record, out_reward, mlp_desc, deterministic, actions_out, logp_out,
                          stream=None):
        """step() into the compact record out_record, fused with the MLP policy of the next slot on that record
        (d2d_comb_policy_fused_step, one launch): actions_out [E][N] and logp_out [N][E] of slot t + 1, drawn at
        the rng_step the two-call sequence (step, then the policy) gives it -- bit-identical results.  mlp_desc:
        an actor-only d2d_mlp_desc on this batch's record (obs_format D2D_OBS_U8)."""
        s = self.spec
        dt = _MASK_DTYPE[s.mask_bytes] if s.kind == COMB else torch.uint8
        self._check_out(actions, (self.E, s.N), dt, "actions")
        self._check_out(actions_out, (self.E, s.N), dt, "actions_out")
        self._check_out(logp_out, (s.N, self.E), torch.float32, "logp_out")
        o, res = self._out(False, False, False, False, out_record, None, out_reward)
        self.timestep += 1
        rc = self.lib.d2d_comb_policy_fused_step(self.desc, self.st, actions.data_ptr(), o, self.timestep,
                                                 self.rng_step, mlp_desc, self.rng_step + 1, 1 if deterministic else 0,
                                                 actions_out.data_ptr(), logp_out.data_ptr(), _lib.stream_ptr(stream))
        _lib.check(rc, "d2d_comb_policy_fused_step")
        self.rng_step += 1
        res["done"] = self.timestep >= s.episode_length
        return res

    def sample_actions(self, p=0.1, out=None, stream=None):
        """Synthetic Philox actions: comb Bernoulli(p) per (agent, channel); chsel uniform id;
        single Bernoulli(p) per agent."""
        a = out if out is not None else self.action_buffer()
        thr = int(np.floor(min(max(p, 0.0), 1.0) * 4294967296.0))
        rc = self.lib.d2d_sample_actions(self.desc, a.data_ptr(), thr, self.rng_step, _lib.stream_ptr(stream))
        _lib.check(rc, "d2d_sample_actions")
        self.rng_step += 1
        return a

    # ------------------------------------------------------- host readback
    def buffers_host(self):
        """[E][N][D] uint8 packet counts (little-endian byte view of the rows)."""
        b = self.buffers.cpu().numpy().view(np.uint8).reshape(self.E, self.spec.N, -1)
        return b[:, :, : self.spec.D]

    def channels_host(self):
        """comb: [E][N][C] uint8; chsel: [E][C+1] uint8; single: [E][N] uint8."""
        s = self.spec
        h = self.channels.cpu().numpy()
        if s.kind == SINGLE:
            return h.astype(np.uint8)
        if s.kind == COMB:
            bits = np.unpackbits(h.view(np.uint8).reshape(self.E, s.N, -1), axis=2, bitorder="little")
            return bits[:, :, : s.C]
        bits = np.unpackbits(h.view(np.uint8).reshape(self.E, -1), axis=1, bitorder="little")
        return bits[:, : s.C + 1]


def pack_masks(bits, n_channels):
    """[..., C] 0/1 array -> little-endian channel masks of d2d_mask_bytes(C) bytes (numpy)."""
    bits = (np.asarray(bits) != 0).astype(np.uint8)
    mb = 1 if n_channels <= 8 else 2 if n_channels <= 16 else 4
    pad = mb * 8 - bits.shape[-1]
    if pad:
        bits = np.concatenate([bits, np.zeros(bits.shape[:-1] + (pad,), dtype=np.uint8)], axis=-1)
    packed = np.packbits(bits, axis=-1, bitorder="little")
    dt = {1: np.uint8, 2: np.int16, 4: np.int32}[mb]
    return np.ascontiguousarray(packed).view(dt)[..., 0]


def pack_masks_torch(bits):
    """[..., C] tensor (0/1 or bool, C <= 32) -> int mask tensor (uint8 / int16 / int32) on the same device."""
    C = bits.shape[-1]
    w = (1 << torch.arange(C, device=bits.device, dtype=torch.int64))
    m = ((bits != 0).to(torch.int64) * w).sum(-1)
    if C <= 8:
        return m.to(torch.uint8)
    if C <= 16:
        return m.to(torch.int32).to(torch.int16)
    return m.to(torch.int32)
