"""Device-resident rollout collection / evaluation shared by iPPO and D2DPPO.

Reference loops replaced (all per agent, per step, batch-1, host<->device
round trips):
  create_rollouts  /root/reference/algorithms/ippo.py:277-343, d2d_ppo.py:279-339
  test             ippo.py:345-388, d2d_ppo.py:341-383
  preprocess_input_for_rnn  ippo.py:390-403, d2d_ppo.py:385-398

Here one slot for all agents of all `env.n_envs` envs is:
  policy forward for all agents (agent-stacked bmm) -> sample -> pack the
  actions into channel masks -> one env-step kernel writing the next obs /
  state straight into the rollout buffers.
Nothing leaves the GPU until an episode ends (scores).

Sequence order: a rollout of E envs x W waves of full episodes is the
reference's sequential rollout of E*W episodes in env-major order
(env 0's episodes, then env 1's, ...); GAE, normalisation and the update
all use that order.
"""
import math
import os

import numpy as np
import torch

from d2dhip.envbatch import pack_masks_torch
from d2dhip.gae import gae_returns
from d2dhip._lib import record_bytes as _lib_record_bytes
from d2dhip.record import ObsRecord, set_format

from ._core import make_dist, rnn_windows, unpack_actions
from .data_parallel import DataParallelMixin, allreduce_mean_scalar


class Rollout:
    """Device tensors of one rollout ([T][E]... time-major as produced).  `adv` / `ret` (agent-
    major [N][E*T], env-major sample order) are materialised from `adv_tne` / `ret_tne`
    ([T][N][E], the GAE output) only when a consumer asks for them; the fused update kernels
    read the [T][N][E] tensors in place.  `obs` is the env kernel's compact record (ObsRecord,
    d2dhip/record.py) when the learner runs on it; `obs_f32` is the fp32 [T][E][N][F] view either way."""

    def __init__(self, **kw):
        self.__dict__.update(kw)

    def __getattr__(self, name):
        if name == "state_seq" and "state_dim" in self.__dict__:
            # env-major fp32 states [E*T][S] (d2d_ppo.py's rollout states), copied from the slot-major
            # buffer only when a consumer asks (the bf16 central critic reads the buffer directly); from the env
            # kernel's bf16 rows (exact integers) when the rollout kept no fp32 copy
            st = self.__dict__.get("states")
            S = self.__dict__["state_dim"]
            if st is None:
                v = self.__dict__["state_bf16"][:, :S].float()
            else:
                v = st[:, :, :S].transpose(0, 1).reshape(st.shape[0] * st.shape[1], -1)
            self.__dict__[name] = v
            return v
        if name == "obs_f32":
            o = self.__dict__["obs"]
            v = o.decode() if isinstance(o, ObsRecord) else o
            self.__dict__[name] = v
            return v
        src = self.__dict__.get(name + "_tne") if name in ("adv", "ret") else None
        if src is None:
            raise AttributeError(name)
        v = src.permute(1, 2, 0).reshape(src.shape[1], -1)
        self.__dict__[name] = v
        return v


class BatchedLearnerBase(DataParallelMixin):
    combinatorial = False
    useRNN = False

    # ------------------------------------------------------------- setup
    def _resolve_device(self, device):
        if device is None:
            dev = torch.device('cuda' if torch.cuda.is_available() else "cpu")
        else:
            dev = torch.device(device)
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        return dev

    def _bind_env(self):
        env = self.env
        if getattr(env, "_batch", None) is None:
            env.device = self.device
        elif env._batch.device != self.device:
            raise ValueError(f"env lives on {env._batch.device}, learner on {self.device}")
        return env.batch()

    @property
    def kind(self):
        return self.env.kind

    def _policy_act(self):
        if self.useRNN:
            return "sigmoid" if self.combinatorial else "softmax"
        return "softmax"  # Policy always ends in softmax (ippo.py:73), Bernoulli of softmax probs (quirk Q6)

    # -------------------------------------------------------- obs plumbing
    def _agent_major(self, obs_t):
        """[E][N][F] -> [N][E][F]"""
        return obs_t.transpose(0, 1)

    def _window(self, obs_buf, ep_start, i):
        """RNN input at step i: last <= history_len obs of the current episode, unpadded
        (ippo.py:302-304), as [N][E][w][F]."""
        lo = max(ep_start, i - self.history_len + 1)
        return obs_buf[lo: i + 1].permute(2, 1, 0, 3)

    def _policy_input(self, obs_buf, ep_start, i):
        if self.useRNN:
            return self._window(obs_buf, ep_start, i)
        return self._agent_major(obs_buf[i])

    def _actions_from_probs(self, probs, train):
        if self.combinatorial:
            if train:
                a = torch.bernoulli(probs)
            else:
                a = (probs > 0.5).to(probs.dtype)
            dist = make_dist(probs, True)
            return a, dist.log_prob(a).mean(-1)
        if train:
            a = torch.multinomial(probs.reshape(-1, probs.shape[-1]), 1).view(probs.shape[:-1])
        else:
            a = probs.argmax(dim=-1)
        dist = make_dist(probs, False)
        return a, dist.log_prob(a)

    # ------------------------------------------------ behaviour policy slot
    def _fused_ok(self):
        """The fused HIP policy kernel covers the MLP policies (A <= 16, F <= 64; H <= 128 with F + 1 <= 32 --
        the learners' default hidden_size 128 on the reference envs -- else H <= 64)."""
        if getattr(self, "_fused", None) is None:
            p = self.policy
            hmax = 128 if p.F + 1 <= 32 else 64
            self._fused = (not self.useRNN and p.kind == "mlp" and p.H <= hmax and p.A <= 16 and p.F <= 64
                           and os.environ.get("D2D_FUSED_POLICY", "1") != "0")
        return self._fused

    def _gru_ok(self):
        """The GRU window-policy kernels (csrc/gru_kernels.hip) cover the RNN learners with H <= 64,
        A <= 16 and F + 1 <= 64 inputs (up to four 16-column input tiles: xp_load's 30 inputs and
        run_ippo_combinatorial.py's 6 x 16-channel env with 14 + 2 * 16 = 46)."""
        if getattr(self, "_gru", None) is None:
            p = self.policy
            self._gru = (self.useRNN and p.kind == "rnn" and p.H <= 64 and p.A <= 16 and p.F + 1 <= 64
                         and (self.kind == "comb") == bool(self.combinatorial)
                         and os.environ.get("D2D_FUSED_POLICY", "1") != "0")
        return self._gru

    def _gru_kind(self):
        return "sigmoid" if self.combinatorial else "softmax"

    # compact obs record (d2dhip/record.py): on by default where every consumer of the rollout's obs
    # is a HIP kernel that reads it; D2D_OBS_RECORD=0 keeps the fp32 obs buffer (A/B timing, tests)
    obs_record = os.environ.get("D2D_OBS_RECORD", "1") != "0"

    def _record_ok(self):
        # the combinatorial env's record, and since round 6 the D2DEnv's (categorical learners; record rows of at most
        # 64 bytes -- the update kernels' F + 1 <= 64 -- and 64 agents, the ring / small neighbourhoods of the drivers)
        s = self.env.spec if self.kind == "single" else None
        env_ok = ((self.kind == "comb" and bool(self.combinatorial))
                  or (self.kind == "single" and not self.combinatorial and s.N <= 64 and _lib_record_bytes(s.F) <= 64))
        return (self.obs_record and env_ok
                and (self._gru_ok() or (not self.useRNN and self._fused_ok())) and self._fused_update_ok())

    def _fused_update_ok(self):
        """The fused HIP update kernels cover the MLP actors with F + 1 <= 64 inputs (and the iPPO
        per-agent MLP critics; csrc/update_kernels.hip) and the GRU policies / critics
        (csrc/gru_kernels.hip)."""
        if getattr(self, "_fused_upd", None) is None:
            self._fused_upd = (((self._fused_ok() and self.policy.F + 1 <= 64) or self._gru_ok())
                               and (self.kind == "comb") == bool(self.combinatorial)
                               and os.environ.get("D2D_FUSED_UPDATE", "1") != "0")
        return self._fused_upd

    @staticmethod
    def _grad_buffers(params):
        """The .grad tensors of agent-stacked params (allocated once; the kernels overwrite them)."""
        for p in params.values():
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        return {k: p.grad for k, p in params.items()}

    def _update_state(self, ro):
        """What an epoch of the update needs beyond the rollout: nothing for the fused kernels
        (they read the rollout buffers in place), the agent-major copies for the torch path."""
        return None if self._fused_update_ok() else self._update_inputs(ro)

    def _logp_forced(self, ro):
        """log-probs of the rollout's own actions under the current actor params, for every
        sample: the policy kernel in forced mode over the T*E slots at once -> [N][T*E] (time-major).
        GRU policies: the training windows (front-zero-padded, ippo.py:390-403)."""
        if self.useRNN:
            from d2dhip import gru
            _, lp = gru.policy({k: v.data for k, v in self.policy.params.items()}, ro.obs, self._gru_kind(),
                               self.history_len, ro.L, 0, ro.T, padded=True, forced=ro.actions,
                               want_actions=False)
            return lp
        from d2dhip import _lib
        lib = _lib.require_gpu()
        N, TE = self.policy.N, ro.T * ro.E
        desc = self._mlp_desc(TE, 0)
        desc.v1 = desc.c1 = desc.v2 = desc.c2 = None
        logp = torch.empty((N, TE), dtype=torch.float32, device=self.device)
        optr = set_format(desc, ro.obs)
        # actions = NULL (ABI 15): forced mode stores only the log-probs (the actions are the input)
        rc = lib.d2d_policy_mlp_step(desc, optr, ro.actions.data_ptr(), 0, 0, None, logp.data_ptr(), None,
                                     _lib.stream_ptr())
        _lib.check(rc, "d2d_policy_mlp_step (forced)")
        return logp

    def _policy_seed(self):
        if getattr(self, "_pseed", None) is None:
            # drawn from torch's global RNG, so torch.manual_seed makes rollouts reproducible,
            # as with the reference's torch.distributions sampling
            self._pseed = int(torch.randint(0, 2 ** 62, (1,)).item())
        return self._pseed

    def _mlp_desc(self, E, env_base, critic=True):
        """critic=False: the actor alone (the kernel's actor-only instantiation: no critic forward where no
        value is stored -- test(), and training rollouts whose values come from the first epoch's critic pass)"""
        from d2dhip import _lib
        p = self.policy.params
        crit = getattr(self, "value", None) if critic else None
        cp = crit.params if (crit is not None and getattr(crit, "kind", None) == "mlp") else None
        ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        return _lib.MlpDesc(self.policy.N, E, self.policy.F, self.policy.H, self.policy.A,
                            0 if self.combinatorial else 1, ptr(p["w1"]), ptr(p["b1"]), ptr(p["w2"]), ptr(p["b2"]),
                            ptr(cp["w1"]) if cp else None, ptr(cp["b1"]) if cp else None,
                            ptr(cp["w2"]) if cp else None, ptr(cp["b2"]) if cp else None,
                            self._policy_seed(), int(env_base))

    gru_carry = os.environ.get("D2D_GRU_CARRY", "1") != "0"

    def _gru_carry(self, b, role, params):
        """The carried-state scratch of one GRU policy on env batch b (None when D2D_GRU_CARRY=0).  Kept with the
        batch it serves (a captured rollout graph bakes in its address); dropped with the batch."""
        if not self.gru_carry:
            return None
        from d2dhip import gru
        cache = self.__dict__.setdefault("_gru_carries", {})
        ent = cache.get(id(b))
        if ent is None or ent[0] is not b:
            ent = cache[id(b)] = (b, {})
        n = gru.carry_floats(params, b.E, self.history_len, self.env.episode_length)
        buf = ent[1].get(role)
        if buf is None or buf.numel() < n:
            buf = ent[1][role] = torch.empty((n,), dtype=torch.float32, device=b.device)
        return buf

    def _policy_slot(self, obs_buf, t0, i, train, act_out, logp_out, val_out, tf, b):
        """Actions for slot i of every env (written to act_out [E][N]), log-probs [N][E], values [N][E]."""
        forced = None if (tf is None or tf["actions"] is None) else tf["actions"][i]
        if self._gru_ok():
            # GRU window policy (+ the iPPO GRU critic): the window of slot i is rebuilt in-kernel from
            # the rollout buffer (unpadded, the last <= history_len obs of the episode, ippo.py:302-304)
            from d2dhip import gru
            E, N = b.E, self.policy.N
            fz = None if forced is None else self._env_actions(forced).contiguous().view(1, E, N)
            # the slots of a wave run in order: while the episode position is below history_len the window extends
            # the previous slot's, whose h the kernel carried (d2d_policy_gru_carry; bitwise the recompute)
            pos = (i - t0) % self.env.episode_length
            carry_in = 1 <= pos < self.history_len
            pp = {k: v.data for k, v in self.policy.params.items()}
            gru.policy(pp, obs_buf, self._gru_kind(),
                       self.history_len, self.env.episode_length, i, 1, padded=False, forced=fz,
                       rng_step=b.rng_step, deterministic=not train, seed=self._policy_seed(),
                       env_base=b.desc.env_base, rng_offset=b.rng_off.data_ptr(), actions_out=act_out.view(1, E, N),
                       out=logp_out, hcarry=self._gru_carry(b, "actor", pp), carry_in=carry_in)
            if val_out is not None:
                cp = {k: v.data for k, v in self.value.params.items()}
                gru.policy(cp, obs_buf, None, self.history_len, self.env.episode_length, i, 1, padded=False,
                           out=val_out, hcarry=self._gru_carry(b, "critic", cp), carry_in=carry_in)
            return act_out
        if self._fused_ok() and (self.kind == "comb") == bool(self.combinatorial):
            from d2dhip import _lib
            lib = _lib.require_gpu()
            desc = self._mlp_desc(b.E, b.desc.env_base, critic=val_out is not None)
            desc.rng_offset = b.rng_off.data_ptr()
            fz = None
            if forced is not None:
                fz = self._env_actions(forced).contiguous()
            optr = set_format(desc, obs_buf[i])
            rc = lib.d2d_policy_mlp_step(desc, optr, None if fz is None else fz.data_ptr(),
                                         b.rng_step, 0 if train else 1, act_out.data_ptr(), logp_out.data_ptr(),
                                         None if val_out is None else val_out.data_ptr(), _lib.stream_ptr())
            _lib.check(rc, "d2d_policy_mlp_step")
            if val_out is not None and desc.v1 is None:
                raise RuntimeError("critic values requested without an MLP critic")
            return act_out
        x = self._policy_input(obs_buf, t0, i)
        a, logp, v = self._act(x, train, val_out is not None, forced)
        logp_out.copy_(logp)
        if val_out is not None:
            val_out.copy_(v)
        act = self._env_actions(a)
        act_out.copy_(act)
        return act_out

    def _act(self, x, train=True, want_values=False, forced=None):
        """One slot of the behaviour policy for all agents and envs: probs -> actions,
        log-probs (ippo.py:154-176 batched) and, for iPPO, the critic values."""
        probs = self.policy.forward(x)
        if forced is None:
            a, logp = self._actions_from_probs(probs, train)
        else:
            a = forced
            dist = make_dist(probs, self.combinatorial)
            logp = dist.log_prob(a).mean(-1) if self.combinatorial else dist.log_prob(a)
        v = self.value.forward(x)[..., 0] if want_values else None
        return a, logp, v

    def _env_actions(self, a):
        """agent-major sampled actions -> env action buffer [E][N]"""
        if self.kind == "comb":
            return pack_masks_torch(a.transpose(0, 1))
        return a.transpose(0, 1).to(torch.uint8).contiguous()

    # ------------------------------------------------------------ rollout
    def _collect(self, num_episodes, train=True, want_values=False, want_state=False, teacher=None):
        """teacher (parity testing): a recorded reference rollout of E * waves episodes,
        dict(actions [E*T][N][C|1] or None, reset_arrivals [E*W][N], flips [E*T][..], arrivals [E*T][N]);
        the env replays the draws, the policy computes probs/log-probs/values of the forced actions
        (or, with actions None, acts itself)."""
        b = self._bind_env()
        if teacher is None and b.E == 1 and num_episodes > 1:
            b = self._episode_batch(num_episodes)
        env = self.env
        E, L = b.E, env.episode_length
        waves = max(1, math.ceil(num_episodes / E))
        if teacher is None and self._graph_ok(train, b, waves * L, want_values, want_state):
            ro = self._collect_graph(b, waves, want_values, want_state)
        else:
            bufs = self._rollout_buffers(b, waves, want_values, want_state)
            tf = self._teacher_tensors(teacher, b, waves) if teacher is not None else None
            self._waves(bufs, b, waves, train, tf)
            ro = self._rollout_result(bufs, b, waves, train)
        self._sync_episode_rng(b)
        return ro

    # ---------------------------------------------- episode-parallel rollouts (n_envs == 1)
    episode_parallel = os.environ.get("D2D_EPISODE_PARALLEL", "1") != "0"

    EPISODE_ENV_BASE = 1 << 31  # Philox env indices of the episode batches (the counter word is 32 bits)

    def _episode_batch(self, n):
        """The reference drivers build their envs with the default n_envs = 1 and roll out
        num_episodes episodes one after another (create_rollouts ippo.py:283, test ippo.py:353).  The
        episodes are independent, so here they run side by side: a private device batch of n envs with
        the env's parameters replaces the n sequential waves.  Single process only (data-parallel ranks
        shard their envs explicitly); D2D_EPISODE_PARALLEL=0 keeps the sequential waves.

        Fresh draws for every episode, as the reference's one global RNG stream gives: the batches'
        Philox env indices start at 2^31 (disjoint from the env's own batch, whose indices start at its
        env_base < 2^31), and every episode batch — the training and the test sizes, and a batch
        rebuilt after eviction — continues ONE learner-level rng_step counter (`_sync_episode_rng`), so
        no two rollouts of the learner draw the same (env index, rng_step) Philox counters."""
        main = self.env.batch()
        if not self.episode_parallel or getattr(self, "world_size", 1) > 1:
            return main
        cache = self.__dict__.setdefault("_episode_batches", {})
        b = cache.get(n)
        if b is None:
            from d2dhip.envbatch import EnvBatch
            if len(cache) >= 2:  # the training and the test batch sizes of a driver
                old = cache.pop(next(iter(cache)))
                self._drop_graphs_of(old)
            if main.desc.env_base + main.E > self.EPISODE_ENV_BASE:
                raise ValueError("the env's own Philox env range overlaps the episode batches' (2^31)")
            b = EnvBatch(main.spec, n, main.device, seed=main.desc.seed, env_base=self.EPISODE_ENV_BASE)
            cache[n] = b
        b.rng_step = self.__dict__.get("_episode_rng_step", 0)
        return b

    def _sync_episode_rng(self, b):
        """After a rollout on an episode batch: the learner-level counter moves past its draws."""
        if b in self.__dict__.get("_episode_batches", {}).values():
            self._episode_rng_step = b.rng_step

    def _drop_graphs_of(self, b):
        """Captured rollout graphs bake in a batch's buffers: drop those of an evicted batch."""
        graphs = self.__dict__.get("_rollout_graphs", {})
        for k in [k for k, G in graphs.items() if G["batch"] is b]:
            del graphs[k]
        carries = self.__dict__.get("_gru_carries", {})
        if id(b) in carries and carries[id(b)][0] is b:
            del carries[id(b)]

    # ------------------------------------------------- rollout body (eager or captured)
    def _rollout_buffers(self, b, waves, want_values, want_state):
        s, E, L, dev = b.spec, b.E, self.env.episode_length, self.device
        T = waves * L
        f64 = lambda: torch.zeros((waves, E), dtype=torch.float64, device=dev)  # noqa: E731
        obs = b.record_buffer((T,)) if self._record_ok() else torch.empty((T, E, s.N, s.F), dtype=torch.float32,
                                                                         device=dev)
        return dict(obs=obs,
                    act=torch.empty((T, E, s.N), dtype=b.action_buffer().dtype, device=dev),
                    logp=torch.empty((T, s.N, E), dtype=torch.float32, device=dev),
                    rew=torch.empty((T, E), dtype=torch.int32, device=dev),
                    val=torch.empty((T, s.N, E), dtype=torch.float32, device=dev) if want_values else None,
                    state=(torch.empty((T, E, s.state_stride), dtype=torch.float32, device=dev)
                           if want_state and want_state != "bf16" else None),
                    # want_state "bf16": the env kernel's exact bf16 rows, env-major [E][T][S8] (the D2D central
                    # critic's operand as it is, no fp32 copy and no conversion pass)
                    state_b=(torch.empty((E, T, -(-s.S // 8) * 8), dtype=torch.bfloat16, device=dev)
                             if want_state == "bf16" else None),
                    recv=f64(), disc=f64(), eprew=f64(), jains=f64(), ch=f64())

    def _waves(self, bufs, b, waves, train, tf):
        """The rollout proper: per wave one reset and L slots of (policy kernel, env kernel), then
        the wave's episode statistics as device reductions (no host synchronisation)."""
        env, s = self.env, b.spec
        L = env.episode_length
        obs_buf, act_buf, logp_buf, rew_i32 = bufs["obs"], bufs["act"], bufs["logp"], bufs["rew"]
        val_buf, state_buf, state_b = bufs["val"], bufs["state"], bufs["state_b"]
        want_state = state_buf is not None or state_b is not None
        s.arrival_kinds()  # the reference's reset-time validation (ValueError / AssertionError)
        with torch.no_grad():
            for w in range(waves):
                t0 = w * L
                b.reset(want_obs=True, want_state=state_buf is not None, out_obs=obs_buf[t0],
                        out_state=state_buf[t0] if state_buf is not None else None,
                        replay_arrivals=None if tf is None else tf["reset_arrivals"][w],
                        out_state_bf16=None if state_b is None else state_b[:, t0])
                fused = self._fused_slot_ok(b, obs_buf, val_buf, want_state, tf)
                if fused:
                    self._fused_slots(b, obs_buf, act_buf, logp_buf, rew_i32, t0, L, train)
                for t in range(0 if fused else L):
                    i = t0 + t
                    act = self._policy_slot(obs_buf, t0, i, train, act_buf[i], logp_buf[i],
                                            val_buf[i] if val_buf is not None else None, tf, b)
                    last = t + 1 == L
                    b.step(act, want_obs=not last, want_state=state_buf is not None and not last,
                           out_obs=None if last else obs_buf[i + 1],
                           out_state=None if (last or state_buf is None) else state_buf[i + 1],
                           out_reward=rew_i32[i], replay=None if tf is None else tf["replay"][i],
                           out_state_bf16=None if (last or state_b is None) else state_b[:, i + 1])
                env.timestep = b.timestep
                bufs["recv"][w].copy_(b.received.sum(1))
                bufs["disc"][w].copy_(b.discarded.sum(1))
                bufs["eprew"][w].copy_(rew_i32[t0:t0 + L].sum(0))
                if not train:
                    bufs["jains"][w].copy_(self._jains_dev(b))
                    if s.kind == "single":  # D2DEnv.channel_errors of the episode (env.py:144-145)
                        bufs["ch"][w].copy_(b.sel_quality)

    # ------------------------------------------ fused env + policy slots
    fused_slot = os.environ.get("D2D_FUSED_SLOT", "0") == "1"

    def _fused_slot_ok(self, b, obs_buf, val_buf, want_state, tf):
        """D2D_FUSED_SLOT=1 (A/B, off by default: tools/gpu/fused_slot.py): the slots of a wave as
        one launch each of the env step fused with the next slot's policy (d2d_comb_policy_fused_step), where
        the prototype covers the rollout: the MLP actor alone (no per-slot values, no states, no teacher) on
        the record of the combinatorial env with 64 agents x 8 channels, hidden <= 64."""
        s = b.spec
        return (self.fused_slot and tf is None and val_buf is None and not want_state
                and isinstance(obs_buf, ObsRecord) and not self.useRNN and self._fused_ok()
                and self.kind == "comb" and bool(self.combinatorial) and s.N == 64 and s.C == 8
                and _lib_record_bytes(s.F) == 32 and self.policy.H <= 64)

    def _fused_slots(self, b, obs_buf, act_buf, logp_buf, rew_i32, t0, L, train):
        """Slot t0 on the policy kernel, then L - 1 fused (env step t, policy t + 1) launches, then the last
        env step: the launches and Philox counters of the two-kernel loop, bit-identical results."""
        self._policy_slot(obs_buf, t0, t0, train, act_buf[t0], logp_buf[t0], None, None, b)
        desc = self._mlp_desc(b.E, b.desc.env_base, critic=False)
        desc.rng_offset = b.rng_off.data_ptr()
        set_format(desc, obs_buf[t0])
        for t in range(L - 1):
            i = t0 + t
            b.step_policy_fused(act_buf[i], obs_buf[i + 1], rew_i32[i], desc, not train, act_buf[i + 1],
                                logp_buf[i + 1])
        b.step(act_buf[t0 + L - 1], want_obs=False, out_reward=rew_i32[t0 + L - 1])

    def _rollout_result(self, bufs, b, waves, train):
        L = self.env.episode_length
        T = waves * L
        # per-episode statistics are [waves][E] on the device; episodes are listed env-major
        # (env 0's waves, then env 1's, ...) like the samples (module docstring)
        em = lambda t: t.t().reshape(-1)  # noqa: E731
        recv, disc = em(bufs["recv"]).cpu(), em(bufs["disc"]).cpu()
        scores = (1 - disc / recv).tolist()
        ep_rewards = em(bufs["eprew"]).cpu().tolist()
        jains = em(bufs["jains"]).cpu().tolist() if not train else []
        ch_errors = em(bufs["ch"]).cpu().tolist() if (not train and b.spec.kind == "single") else []
        dones = torch.zeros(T, dtype=torch.uint8, device=self.device)
        dones[L - 1::L] = 1
        ro = Rollout(obs=bufs["obs"], actions=bufs["act"], logp=bufs["logp"], rewards=bufs["rew"].float(),
                     values=bufs["val"], states=bufs["state"], dones=dones, scores=scores, ep_rewards=ep_rewards,
                     jains=jains, ch_errors=ch_errors, T=T, E=b.E, waves=waves, L=L)
        if bufs["state_b"] is not None:
            sb = bufs["state_b"]
            ro.state_bf16 = sb.view(sb.shape[0] * sb.shape[1], sb.shape[2])  # [E*T][S8], env-major samples
        return ro

    # ------------------------------------------------------- HIP-graph rollout
    graph_rollout = os.environ.get("D2D_GRAPH_ROLLOUT", "1") != "0"
    GRAPH_ROLLOUT_MAX_BYTES = 40 << 30

    def _graph_ok(self, train, b, T, want_values=False, want_state=False):
        """Training rollouts of the fused MLP policy replay one captured HIP graph (reset + L x
        (policy kernel, env kernel) per wave + the statistics): at small batches the slot loop is
        bound by per-launch host work, not the GPU.  The graph keeps its rollout buffers alive for the
        learner's lifetime (reused by every replay), so all of them — obs (record or fp32 rows), actions,
        log-probs, values, rewards and D2D-PPO's [T][E][state_stride] fp32 states — count against a
        40 GiB budget (of the 288 GB HBM); larger rollouts stay eager.  The compact record puts the
        headline iPPO rollout inside: 65,536 envs x 200 slots x 64 agents x (32 B record + 1 B actions
        + 4 B log-prob + 4 B value) = 34.4 GB."""
        if not (self.graph_rollout and train and (self._gru_ok() or (not self.useRNN and self._fused_ok()))
                and (self.kind == "comb") == bool(self.combinatorial)):
            return False
        s = b.spec
        row = _lib_record_bytes(s.F) if self._record_ok() else 4 * s.F
        act = b.action_buffer().element_size()
        per_slot_agent = row + act + 4 + (4 if want_values else 0)
        state_row = (2 * (-(-s.S // 8) * 8) if want_state == "bf16" else 4 * s.state_stride) if want_state else 0
        per_slot_env = s.N * per_slot_agent + 4 + state_row
        return T * b.E * per_slot_env <= self.GRAPH_ROLLOUT_MAX_BYTES

    def _collect_graph(self, b, waves, want_values, want_state):
        """Capture once per rollout shape, replay afterwards.  The kernels add the device word
        b.rng_off to their launch's rng_step, so a replay draws the Philox counters an eager rollout
        from the current b.rng_step would (bit-identical results); its buffers are reused by the next
        training rollout of the same shape."""
        env = self.env
        L = env.episode_length
        # the graph bakes in the env batch's state buffers and the stacked parameters' addresses; the
        # entry holds the batch itself (so its buffers outlive the graph) and must be THIS batch — a
        # new batch could reuse a freed one's id()
        key = (id(b), b.E, L, waves, bool(want_values), want_state or False,
               tuple(t.data_ptr() for t in self.policy.params.values()),
               tuple(t.data_ptr() for t in getattr(self.value, "params", {}).values()) if hasattr(self, "value") else ())
        cache = self.__dict__.setdefault("_rollout_graphs", {})
        G = cache.get(key)
        if G is not None and G["batch"] is not b:
            G = None
        if G is None:
            cache.clear()  # one live graph (and its buffers) per learner
            bufs = self._rollout_buffers(b, waves, want_values, want_state)
            side = torch.cuda.Stream(device=self.device)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):  # warm-up: a real rollout (allocations, kernel attributes)
                self._waves(bufs, b, waves, True, None)
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize(self.device)
            result = self._rollout_result(bufs, b, waves, True)
            base, ts = b.rng_step, b.timestep
            g = torch.cuda.CUDAGraph()
            try:
                # thread_local: other threads' runtime calls (e.g. a process group's watchdog
                # querying its events) do not invalidate this thread's capture
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    self._waves(bufs, b, waves, True, None)
            except RuntimeError as err:  # capture unsupported here: keep the eager slot loop
                b.rng_step, b.timestep = base, ts
                self.graph_rollout = False
                print(f"[d2d] rollout graph capture failed ({err}); eager rollouts from now on")
                return result
            G = dict(graph=g, bufs=bufs, base=base, delta=b.rng_step - base, batch=b)
            b.rng_step = base  # capturing ran nothing
            cache[key] = G
            return result
        b.rng_off.fill_(b.rng_step - G["base"])
        G["graph"].replay()
        b.rng_off.zero_()
        b.rng_step += G["delta"]
        b.timestep = L
        env.timestep = L
        return self._rollout_result(G["bufs"], b, waves, True)

    def _teacher_tensors(self, teacher, b, waves):
        """Per-slot device tensors of a recorded reference rollout of E * waves sequential episodes.
        Reference episode q = e * waves + w is replayed by env e in wave w (the env-major sample order
        of _collect), so slot i = w * L + t of env e takes reference step (e * waves + w) * L + t.
        teacher["actions"] may be None (test(): the policy acts deterministically on its own)."""
        from d2dhip.envbatch import pack_masks
        s, dev, E, L = b.spec, b.device, b.E, self.env.episode_length
        T = waves * L
        need = E * T
        fl_all = np.asarray(teacher["flips"])
        if fl_all.shape[0] < need or len(teacher["reset_arrivals"]) < E * waves:
            raise ValueError(f"teacher holds {fl_all.shape[0]} steps; {E} envs x {waves} waves need {need}")
        # reference step index of (slot i, env e)
        ref = (np.arange(E)[None, :] * waves + (np.arange(T) // L)[:, None]) * L + (np.arange(T) % L)[:, None]
        a = None
        if teacher.get("actions") is not None:
            acts = np.asarray(teacher["actions"], dtype=np.float64)[ref]                   # [T][E][...]
            if self.combinatorial:
                a = torch.from_numpy(acts.reshape(T, E, s.N, -1).transpose(0, 2, 1, 3).astype(np.float32))
            else:
                a = torch.from_numpy(acts.reshape(T, E, s.N).transpose(0, 2, 1).astype(np.int64))
            a = a.contiguous().to(dev)                                                      # [T][N][E](...)
        fl = fl_all[ref]                                                                    # [T][E][...]
        arr = np.asarray(teacher["arrivals"])[ref].astype(np.uint8)                         # [T][E][N]
        replay = []
        for i in range(T):
            if s.kind == "comb":
                f = torch.from_numpy(np.ascontiguousarray(pack_masks(fl[i], s.C))).to(dev)
            elif s.kind == "single":
                f = torch.from_numpy(np.ascontiguousarray(fl[i].reshape(E, s.N).astype(np.uint8))).to(dev)
            else:
                words = (fl[i].astype(np.int64) << np.arange(fl[i].shape[-1])).sum(-1)
                f = torch.from_numpy(words.astype(np.int32)).to(dev)
            replay.append((f, torch.from_numpy(np.ascontiguousarray(arr[i])).to(dev)))
        ra_all = np.asarray(teacher["reset_arrivals"], dtype=np.uint8)
        ra = [torch.from_numpy(np.ascontiguousarray(ra_all[np.arange(E) * waves + w])).to(dev) for w in range(waves)]
        return {"actions": a, "replay": replay, "reset_arrivals": ra}

    @staticmethod
    def _jains_dev(b):
        recv = b.received.double()
        disc = b.discarded.double()
        u = torch.where(recv > 0, 1 - disc / recv.clamp(min=1), torch.ones_like(recv))
        return u.sum(1) ** 2 / recv.shape[1] / (u ** 2).sum(1)

    # ------------------------------------------------------ update inputs
    def _seq(self, x_tne):
        """[T][N][E] -> [N][E*T] (env-major sample order)"""
        return x_tne.permute(1, 2, 0).reshape(x_tne.shape[1], -1)

    def _update_inputs(self, ro):
        """Agent-major update tensors from a rollout."""
        s = self.env.batch().spec
        N = s.N
        if self.useRNN:
            seq = ro.obs_f32.permute(1, 2, 0, 3).reshape(ro.E * N, ro.T, -1)      # [E*N][T][F]
            win = rnn_windows(seq, self.history_len, ro.L)                        # [E*N][T][L][F]
            x = win.view(ro.E, N, ro.T, self.history_len, -1).transpose(0, 1).reshape(N, ro.E * ro.T,
                                                                                       self.history_len, -1)
        else:
            x = ro.obs_f32.permute(2, 1, 0, 3).reshape(N, ro.E * ro.T, -1)
        acts = ro.actions.permute(2, 1, 0).reshape(N, -1)                        # [N][E*T]
        if self.kind == "comb":
            acts = unpack_actions(acts, s.C)                                      # [N][B][C]
        else:
            acts = acts.long()
        return x, acts, self._seq(ro.logp)

    def _evaluate(self, x, acts):
        probs = self.policy.forward(x)
        dist = make_dist(probs, self.combinatorial)
        if self.combinatorial:
            return dist.log_prob(acts).mean(-1), dist.entropy().mean(-1)
        return dist.log_prob(acts), dist.entropy()

    # ------------------------------------------------------------- test
    def test(self, num_episodes):
        """Deterministic evaluation (ippo.py:345-388, d2d_ppo.py:341-383): argmax / p > 0.5 actions,
        returns (mean URLLC score, mean Jain's index, summed channel errors, mean episode reward)."""
        return self._test(num_episodes)

    def _test(self, num_episodes, teacher=None):
        """test() body; `teacher` (parity tests) replays recorded env draws, actions stay the policy's."""
        ro = self._collect(num_episodes, train=False, teacher=teacher)
        self._last_test_rollout = ro if teacher is not None else None
        n = num_episodes
        sc = np.array(ro.scores[:n], dtype=np.float64)
        ja = np.array(ro.jains[:n], dtype=np.float64)
        rw = np.array(ro.ep_rewards[:n], dtype=np.float64)
        # channel_errors is never incremented by the comb / chsel envs (combinatorial_env.py:97);
        # the D2DEnv counts failed single attempts (env.py:144-145), summed over episodes (ippo.py:385-388)
        ch = float(np.sum(ro.ch_errors[:n])) if ro.ch_errors else 0
        out = [np.mean(sc), np.mean(ja), ch, np.mean(rw)]
        if getattr(self, "world_size", 1) > 1:  # every rank must take the same save / early-stop branch
            out = [allreduce_mean_scalar(v, self.device, self.process_group) for v in out]
            out[2] = out[2] * self.world_size  # channel errors are a sum over every rank's episodes
        return tuple(out)

    # --------------------------------------------------------- save/load
    def save(self, checkpoint_path):
        if getattr(self, "rank", 0) != 0:
            return
        for i, agent in enumerate(self.agents):
            sd = {k: v.detach().clone().cpu() for k, v in agent.policy_network.state_dict().items()}
            torch.save(sd, f"{checkpoint_path}/agent_{i}.pth")
        print("Models saved!")

    def load(self, checkpoint_path):
        for i, agent in enumerate(self.agents):
            sd = torch.load(f"{checkpoint_path}/agent_{i}.pth", map_location=self.device, weights_only=True)
            agent.policy_network.load_state_dict(sd)
        print("Models loaded!")

    def preprocess_input_for_rnn(self, obs_agent):
        """(T, in) -> (T, history_len, in), front-zero-padded per episode (ippo.py:390-403)."""
        return rnn_windows(obs_agent.unsqueeze(0), self.history_len, self.env.episode_length)[0]

    # ----------------------------------------------------- GAE wrapper
    def _gae(self, rewards_te, values_tec, dones, normalize_adv=True, normalize_ret=True, layout="tec"):
        return gae_returns(rewards_te, values_tec, dones, self.gamma, 0.97, normalize_adv=normalize_adv, layout=layout,
                           normalize_ret=normalize_ret, group=self.process_group,
                           last_shard=self._last_shard(), n_envs_total=self._n_envs_total())

    process_group = None  # set by DataParallelMixin._setup_data_parallel when world_size > 1

    # ------------------------------------------------------------ phase marks
    phase_timer = None  # bench.py installs one to split an iteration into phases (stream events)

    def _phase(self, name):
        """Attribute the GPU time since the previous mark to `name` (no-op unless timed)."""
        t = self.phase_timer
        if t is not None:
            t.mark(name)
