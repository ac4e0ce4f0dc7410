"""Shared host side of the two device-backed envs.

Keeps the reference's duck-typed env protocol — attributes,
reset()/step() return structures, metric methods — while every slot runs as
one HIP kernel over E = n_envs environments (d2dhip.EnvBatch).

n_envs == 1 (default): reset/step return exactly the reference's Python
structures (lists of float64 numpy arrays, int64 reward vector, bool done).
n_envs  > 1: the same structures with a leading env axis on every array, and
the learners use the zero-copy device API (reset_batched / step_batched).
"""
import numpy as np

from d2dhip.spec import COMB, EnvSpec


def _default_seed():
    # drawn from the legacy global numpy stream so `np.random.seed(s)` in a
    # driver (xp_load.py:14) keeps runs reproducible
    hi, lo = np.random.randint(0, 2 ** 31, size=2)
    return (int(hi) << 31) | int(lo)


class DeviceEnvBase:
    kind = None

    def _init_common(self, n_envs, device, seed):
        self.n_envs = int(n_envs)
        if self.n_envs < 1:
            raise ValueError("n_envs must be >= 1")
        self.device = device
        self.seed = _default_seed() if seed is None else int(seed)
        self.env_base = 0
        self._batch = None
        self._spec = None
        self.timestep = 0
        self.last_attempts = 0
        self.successful_transmissions = 0
        self.last_feedback = 0
        self.channel_errors = 0
        self.n_collisions = 0
        self.last_time_transmitted = np.ones(self.n_agents) if self.n_envs == 1 else np.ones((self.n_envs, self.n_agents))

    # ----------------------------------------------------------- plumbing
    def _make_spec(self):
        raise NotImplementedError

    @property
    def spec(self):
        if self._spec is None:
            self._spec = self._make_spec()
        return self._spec

    def batch(self):
        """The device EnvBatch (created on first use, like the reference's reset-time validation)."""
        if self._batch is None:
            from d2dhip.envbatch import EnvBatch
            import torch
            dev = self.device
            if dev is None:
                dev = "cuda"
            dev = torch.device(dev)
            if dev.type == "cuda" and dev.index is None:
                dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else dev
            self._batch = EnvBatch(self.spec, self.n_envs, dev, self.seed, self.env_base)
        return self._batch

    def shard(self, rank, world_size, n_envs_global=None):
        """Make this env the `rank`-th contiguous shard of a global batch (distinct Philox streams)."""
        if self._batch is not None:
            raise RuntimeError("shard() must be called before the first reset")
        self.env_base = int(rank) * self.n_envs
        return self

    # ---------------------------------------------------- batched device API
    def reset_batched(self, want_obs=True, want_state=False, **kw):
        b = self.batch()
        self.spec.arrival_kinds()  # reference-equivalent validation (ValueError / AssertionError)
        out = b.reset(want_obs=want_obs, want_state=want_state, **kw)
        self.timestep = 0
        return out

    def step_batched(self, actions, want_obs=True, want_state=False, **kw):
        out = self.batch().step(actions, want_obs=want_obs, want_state=want_state, **kw)
        self.timestep = self._batch.timestep
        return out

    # ------------------------------------------------ reference numpy API
    def _validate_reset(self):
        self.spec.arrival_kinds()

    def reset(self):
        self._validate_reset()
        b = self.batch()
        out = b.reset(want_obs=True, want_state=True)
        self.timestep = 0
        self.last_attempts = 0
        self.successful_transmissions = 0
        self.last_feedback = 0
        self.channel_errors = 0
        self.n_collisions = 0
        self.last_time_transmitted[...] = 1
        obs = out["obs"].cpu().numpy()
        state = out["state"].cpu().numpy()
        return self._ref_obs(obs, None), self._ref_state(state, None, reset=True)

    def step(self, actions):
        s = self.spec
        b = self.batch()
        a = self._pack_actions(actions)
        out = b.step(a, want_obs=True, want_state=True, want_ack=True, want_success=True)
        self.timestep = b.timestep
        self.last_time_transmitted += 1
        self.last_attempts += 1
        reward = out["reward"].cpu().numpy().astype(np.int64)
        succ = out["success"].cpu().numpy().astype(bool)
        ack = out["ack"].cpu().numpy().astype(np.float64)
        obs = out["obs"].cpu().numpy()
        state = out["state"].cpu().numpy()
        if self.n_envs == 1:
            self.last_time_transmitted[succ[0]] = 1.0
            self.successful_transmissions += int(reward[0])
            self.last_feedback = ack[0]
            rewards = np.full(s.N, reward[0], dtype=np.int64)
        else:
            self.last_time_transmitted[succ] = 1.0
            self.successful_transmissions = self.successful_transmissions + reward
            self.last_feedback = ack
            rewards = np.repeat(reward[:, None], s.N, axis=1)
        if self.verbose:
            print(f"Timestep {self.timestep}")
            print(f"ACK/NACK {self.last_feedback}")
            print(f"Reward {rewards}")
            print(f"Received packets {self.received_packets}")
            print(f"Number of discarded packets {self.discarded_packets.sum()}")
            print("")
        done = self.timestep >= s.episode_length
        return self._ref_obs(obs, ack), self._ref_state(state, ack, reset=False), rewards, done, {}

    # reference structures from the device layout
    def _ref_obs(self, obs, ack):
        s = self.spec
        out = []
        for k in range(s.N):
            o = obs[:, k, : s.obs_len[k]].astype(np.float64)
            if s.kind != COMB and ack is not None:
                o[:, s.w[k]:] = ack  # exact float64 1/n feedback (channel_selection_env.py:137)
            out.append(o[0] if self.n_envs == 1 else o)
        return out

    def _ref_state(self, state, ack, reset):
        s = self.spec
        st = state[:, : s.S].astype(np.float64)
        nb = int(s.d.sum())
        if s.kind == COMB:
            parts = [st[:, :nb], st[:, nb: nb + s.N * s.C], st[:, nb + s.N * s.C:]]
        else:
            parts = [st[:, :nb], st[:, nb:]]
        return [p[0] for p in parts] if self.n_envs == 1 else parts

    # ------------------------------------------------------ host readback
    def _host(self, t):
        v = t.cpu().numpy().astype(np.float64)
        return v[0] if self.n_envs == 1 else v

    @property
    def received_packets(self):
        if self._batch is None:
            raise AttributeError("received_packets is defined after reset()")
        return self._host(self._batch.received)

    @property
    def discarded_packets(self):
        if self._batch is None:
            raise AttributeError("discarded_packets is defined after reset()")
        return self._host(self._batch.discarded)

    @property
    def current_buffers(self):
        b = self.batch().buffers_host().astype(np.float64)
        return b[0] if self.n_envs == 1 else b

    @property
    def channel_state(self):
        h = self.batch().channels_host().astype(np.float64)
        return h[0] if self.n_envs == 1 else h

    # ---------------------------------------------------------- metrics
    def _urllc_per_agent(self):
        recv = np.atleast_2d(self.received_packets)
        disc = np.atleast_2d(self.discarded_packets)
        with np.errstate(divide="ignore", invalid="ignore"):
            return np.where(recv > 0, 1 - disc / np.where(recv > 0, recv, 1), 1.0)

    def compute_jains(self):
        """Jain's index of per-agent URLLC scores (combinatorial_env.py:245-254)."""
        u = self._urllc_per_agent()
        j = u.sum(1) ** 2 / self.n_agents / (u ** 2).sum(1)
        return j[0] if self.n_envs == 1 else j

    def compute_urllc(self):
        """1 - discarded / received (combinatorial_env.py:256-258)."""
        recv = np.atleast_2d(self.received_packets)
        disc = np.atleast_2d(self.discarded_packets)
        v = 1 - disc.sum(1) / recv.sum(1)
        return v[0] if self.n_envs == 1 else v

    def compute_channel_score(self):
        """selected_channel_qualities / number_selected_channel (1 if none), combinatorial_env.py:260-264."""
        q = np.atleast_1d(self.selected_channel_qualities).astype(np.float64)
        n = np.atleast_1d(self.number_selected_channel).astype(np.float64)
        v = np.where(n != 0, q / np.where(n != 0, n, 1), 1)
        return v[0] if self.n_envs == 1 else v


def make_spec(kind, env):
    return EnvSpec(kind, env.n_agents, env.n_channels, env.deadlines, env.lbdas, env.period, env.arrival_probs,
                   env.offsets, env.episode_length, env.traffic_model, env.periodic_devices,
                   getattr(env, "homogeneous_size", False), env.channel_switch)
