"""TEST INFRASTRUCTURE ONLY — the CPU checker for the HIP env kernels.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module; the product path (d2d-ppo_amd/) never imports it.

A plain numpy restatement of the reference environments, one env at a time,
following the reference's own control flow line by line:

  CombinatorialEnv    /root/reference/envs/combinatorial_env.py
      reset 61-114, evolve_channel 116-118, evolve_buffer 120-124,
      step 127-242, compute_jains 245-254, compute_urllc 256-258
  ChannelSelectionEnv /root/reference/envs/channel_selection_env.py
      reset 49-98, evolve_channel 104-107, evolve_buffer 109-113,
      step 116-214, metrics 217-236
  D2DEnv ("single")   /root/reference/envs/env.py
      reset 51-99, decode_signal 101-103, evolve_channel 105-107,
      evolve_buffer 109-113, step 116-213, metrics 216-233

Randomness comes from one of two sources:
  * replay  — the draws recorded from the reference (tests/golden/env_*.npz):
              per step the channel-flip mask and the per-agent arrival value;
  * philox  — this framework's production stream (oracle/philox.py).
Pinned by tests/test_oracle_golden.py against every golden env fixture.

Output layout (shared with the HIP kernels):
  obs   [E][N][F]  agent k's row = [B[k,:w_k], chan_obs, ack, 0...]   (prefix-compact)
        comb:  w_k = D if homogeneous_size else d_k, F = D + 2C
        chsel: w_k = d_k, F = D + C + 1
        single: [B[j,:d_j] for j in nbr(k)], H[nbr(k)] (post-evolve), ack, 0...;
                F = max_k (sum_{j in nbr(k)} d_j + |nbr(k)| + 1)
  state [E][S]     the reference's np.concatenate(state)
"""
import numpy as np

from . import philox


def _as_array(x, n=None, dtype=np.float64):
    a = np.asarray(x, dtype=dtype)
    if n is not None and a.ndim == 0:
        a = np.full(n, a, dtype=dtype)
    return a


class _Spec:
    """Per-agent tables derived from the reference constructor kwargs."""

    def __init__(self, kind, n_agents, deadlines, lbdas, n_channels=1, period=5, arrival_probs=None, offsets=None,
                 episode_length=100, traffic_model="aperiodic", periodic_devices=(), homogeneous_size=False,
                 channel_switch=None, neighbourhoods=None, **_ignored):
        self.kind = kind
        N, C = int(n_agents), int(n_channels)
        self.N, self.C = N, C
        self.d = np.asarray(deadlines, dtype=np.int64)
        self.D = int(self.d.max())
        self.homog = bool(homogeneous_size) and kind == "comb"
        self.w = np.full(N, self.D) if self.homog else self.d.copy()
        self.episode_length = episode_length
        self.traffic_model = traffic_model
        pdev = [int(i) for i in np.asarray(periodic_devices).reshape(-1)] if periodic_devices is not None else []
        self.periodic_devices = pdev
        self.aperiodic_devices = [i for i in range(N) if i not in pdev]
        self.lam = _as_array(lbdas, N) if lbdas is not None else np.zeros(N)
        self.q = _as_array(arrival_probs, N) if arrival_probs is not None else np.zeros(N)
        self.period = _as_array(period, N) if period is not None else np.ones(N)
        self.offsets = _as_array(offsets, N) if offsets is not None else np.zeros(N)
        if kind == "comb":
            cs = np.zeros((N, C)) if channel_switch is None else np.broadcast_to(
                np.asarray(channel_switch, dtype=np.float64), (N, C))
        elif kind == "single":
            # env.py:33, 106: one scalar (or per-agent) flip probability, default 0.2
            cs = np.broadcast_to(np.asarray(0.2 if channel_switch is None else channel_switch, dtype=np.float64), (N,))
        else:
            cs = np.zeros(N) if channel_switch is None else np.asarray(channel_switch, dtype=np.float64)
        self.switch = np.array(cs, dtype=np.float64)
        if kind == "comb":
            self.F = self.D + 2 * C
            self.S = int(self.d.sum()) + C * (N + 1)
        elif kind == "single":
            self.nbr = [[int(k)] for k in range(N)] if neighbourhoods is None else \
                [[int(j) for j in nb] for nb in neighbourhoods]                              # env.py:39-42
            self.obs_len = np.array([int(self.d[nb].sum()) + len(nb) + 1 for nb in self.nbr])   # env.py:44-45
            self.F = int(self.obs_len.max())
            self.S = int(self.d.sum()) + N + 1                                                # env.py:48-49
        else:
            self.F = self.D + C + 1
            self.S = int(self.d.sum()) + C + 1
        self.state_off = np.concatenate([[0], np.cumsum(self.d)[:-1]]).astype(np.int64)

    def arrival_draws(self, t):
        """(agent, 'poisson'|'bernoulli') in the reference's draw order at timestep t
        (reset: t = 0 <=> offsets == 0, combinatorial_env.py:66-85 / 178-196)."""
        tm = self.traffic_model
        if tm == "aperiodic":
            return [(i, "poisson") for i in range(self.N)]
        if tm == "periodic":
            if t == 0:
                act = np.where(self.offsets == 0)[0]
            else:
                act = np.where(np.fmod(float(t), self.period) == self.offsets)[0]
            return [(int(i), "bernoulli") for i in act]
        if tm == "heterogeneous":
            assert len(self.periodic_devices) > 0 and len(self.aperiodic_devices) > 0, \
                "periodic_devices and aperiodic_devices must be non empty"
            out = [(i, "poisson") for i in self.aperiodic_devices]
            for i in self.periodic_devices:
                if (self.offsets[i] == 0) if t == 0 else (np.fmod(float(t), self.period[i]) == self.offsets[i]):
                    out.append((i, "bernoulli"))
            return out
        raise ValueError("traffic model not supported")


class EnvOracle:
    """E independent envs (loop over envs; each env follows the reference step)."""

    def __init__(self, kind, params, n_envs=1, seed=0, env_base=0):
        self.spec = _Spec(kind, **params)
        self.E = int(n_envs)
        self.seed = int(seed)
        self.env_base = int(env_base)
        s = self.spec
        self.buffers = np.zeros((self.E, s.N, s.D), dtype=np.int64)
        self.chan = np.ones((self.E, s.N, s.C) if kind == "comb" else (self.E, s.N) if kind == "single"
                            else (self.E, s.C + 1), dtype=np.int64)
        self.channel_errors = np.zeros(self.E, dtype=np.int64)
        self.n_collisions = np.zeros(self.E, dtype=np.int64)
        self.successful_transmissions = np.zeros(self.E, dtype=np.int64)
        self.received = np.zeros((self.E, s.N), dtype=np.int64)
        self.discarded = np.zeros((self.E, s.N), dtype=np.int64)
        self.sel_q = np.zeros(self.E, dtype=np.int64)
        self.sel_n = np.zeros(self.E, dtype=np.int64)
        self.timestep = 0

    # ----------------------------------------------------------------- draws
    def _arrivals(self, t, rng_step, replay):
        """[E][N] arrival values; replay[e][k] is used as-is for agents that draw."""
        s = self.spec
        out = np.zeros((self.E, s.N), dtype=np.int64)
        draws = s.arrival_draws(t)
        if not draws:
            return out, draws
        if replay is not None:
            for (i, _k) in draws:
                out[:, i] = np.asarray(replay)[:, i]
            return out, draws
        envs = self.env_base + np.arange(self.E, dtype=np.uint64)
        r = philox.words(envs[:, None], np.arange(s.N, dtype=np.uint64)[None, :], rng_step,
                         philox.STREAM_ARRIVAL, 1, self.seed)[..., 0]
        for (i, kind) in draws:
            if kind == "poisson":
                out[:, i] = philox.poisson_inversion(r[:, i], s.lam[i], np.exp(-s.lam[i]))
            else:
                out[:, i] = (r[:, i] < philox.threshold(s.q[i])).astype(np.int64)
        return out, draws

    def _flips(self, rng_step, replay):
        s = self.spec
        if replay is not None:
            return np.asarray(replay, dtype=np.int64)
        envs = self.env_base + np.arange(self.E, dtype=np.uint64)
        if self.kind == "single":  # one word per (env, agent) against the agent's switch threshold
            r = philox.words(envs[:, None], np.arange(s.N, dtype=np.uint64)[None, :], rng_step,
                             philox.STREAM_FLIP, 1, self.seed)[..., 0]
            return (r < philox.threshold(s.switch)[None]).astype(np.int64)
        if self.kind == "comb":
            r = philox.words(envs[:, None], np.arange(s.N, dtype=np.uint64)[None, :], rng_step,
                             philox.STREAM_FLIP, s.C, self.seed)
            return (r < philox.threshold(s.switch)[None]).astype(np.int64)
        r = philox.words(envs, philox.PER_ENV, rng_step, philox.STREAM_FLIP, s.C + 1, self.seed)
        return (r < philox.threshold(s.switch[: s.C + 1])[None]).astype(np.int64)

    @property
    def kind(self):
        return self.spec.kind

    # ------------------------------------------------------------- emission
    def _obs_state(self, chan_obs, ack):
        s = self.spec
        obs = np.zeros((self.E, s.N, s.F), dtype=np.float64)
        state = np.zeros((self.E, s.S), dtype=np.float64)
        if self.kind == "single":
            for e in range(self.E):
                for k in range(s.N):
                    nb = s.nbr[k]
                    row = np.concatenate([self.buffers[e, j, :s.d[j]] for j in nb] + [self.chan[e, nb], ack[e]])
                    obs[e, k, :row.shape[0]] = row                                   # env.py:91-95 / 198-202
                allb = np.concatenate([self.buffers[e, k, :s.d[k]] for k in range(s.N)])
                state[e] = np.concatenate([allb, self.chan[e], ack[e]])              # env.py:97-98 / 204-205
            return obs, state
        for e in range(self.E):
            for k in range(s.N):
                w = s.w[k]
                row = [self.buffers[e, k, :w]]
                if self.kind == "comb":
                    row += [chan_obs[e][k], ack[e]]
                else:
                    row += [ack[e]]
                row = np.concatenate(row)
                obs[e, k, :row.shape[0]] = row
            allb = np.concatenate([self.buffers[e, k, :s.d[k]] for k in range(s.N)])
            if self.kind == "comb":
                state[e] = np.concatenate([allb, self.chan[e].reshape(-1), ack[e]])
            else:
                state[e] = np.concatenate([allb, self.chan[e]])
        return obs, state

    # ---------------------------------------------------------------- reset
    def reset(self, rng_step=0, arrivals=None):
        s = self.spec
        self.buffers[:] = 0
        arr, draws = self._arrivals(0, rng_step, arrivals)
        for (i, _k) in draws:
            self.buffers[:, i, s.d[i] - 1] = arr[:, i]
        self.chan[:] = 1
        self.timestep = 0
        self.discarded[:] = 0
        self.received[:] = self.buffers.sum(2)
        self.sel_q[:] = 0
        self.sel_n[:] = 0
        self.channel_errors[:] = 0
        self.n_collisions[:] = 0
        self.successful_transmissions[:] = 0
        if self.kind == "single":
            obs, state = self._obs_state(None, np.zeros((self.E, 1)))   # last_feedback = 0 (env.py:85)
        elif self.kind == "comb":
            chan_obs = np.ones((self.E, s.N, s.C))
            ack = np.ones((self.E, s.C))   # reset state/obs use ones (combinatorial_env.py:108-112)
            obs, state = self._obs_state(chan_obs, ack)
        else:
            ack = np.zeros((self.E, s.C + 1))   # channel_selection_env.py:93
            obs, state = self._obs_state(None, ack)
        return dict(obs=obs, state=state, buffers=self.buffers.copy(), chan=self.chan.copy(),
                    received=self.received.copy(), arrivals=arr)

    # ----------------------------------------------------------------- step
    def step(self, actions, rng_step=1, flips=None, arrivals=None):
        s = self.spec
        self.timestep += 1
        t = self.timestep
        E, N, C = self.E, s.N, s.C
        actions = np.asarray(actions)
        rewards = np.zeros(E, dtype=np.int64)
        success = np.zeros((E, N), dtype=bool)
        if self.kind == "single":
            return self._step_single(actions, rng_step, flips, arrivals)
        if self.kind == "comb":
            ack = np.zeros((E, C))
        else:
            ack = np.zeros((E, C + 1))
        chan_obs = self.chan.copy()
        nxt = self.buffers.copy()
        for e in range(E):
            has = (self.buffers[e].sum(1) > 0) * 1                                  # 135 / 124
            if self.kind == "comb":
                att = (actions[e] != 0).astype(np.int64) * has[:, None]            # 136-137
                good = att * self.chan[e]                                           # 138
                n_c = att.sum(0)                                                    # 148
                a = np.zeros(C) - 1                                                 # 155
                a[(good.sum(0) == 1) & (n_c == 1)] = 1                              # 156
                a[n_c == 0] = 0                                                     # 157
                succ_att = (a[None, :] * good) == 1                                 # 160
                users = np.unique(succ_att.nonzero()[0])                            # 161
            else:
                att = actions[e].astype(np.int64) * has                             # 125
                idx, counts = np.unique(att[att != 0], return_counts=True)          # 127
                a = np.zeros(C + 1)
                a[idx] = 2 * self.chan[e][idx] - 1                                  # 131
                self.sel_q[e] += (a > 0).sum()                                      # 132
                self.sel_n[e] += (a != 0).sum()                                     # 133
                goodmask = self.chan[e][idx] != 0
                a[idx[goodmask]] = 1 / counts[goodmask]                             # 136-137
                g1 = idx[counts == 1]
                g1 = g1[self.chan[e][g1] == 1]                                      # 140-141
                users = np.where(np.isin(att, g1))[0]                               # 142
            ack[e] = a
            for u in users:                                                         # 164-170 / 145-151
                col = nxt[e, u].nonzero()[0]
                nxt[e, u, col.min()] -= 1
                success[e, u] = True
            rewards[e] = len(users)                                                 # 211 / 188
        expired = nxt[:, :, 0].copy()                                               # 120-124 / 109-113
        nxt = np.concatenate([nxt[:, :, 1:], np.zeros((E, N, 1), dtype=np.int64)], axis=2)
        self.discarded += expired
        F = self._flips(rng_step, flips)                                            # 116-118 / 104-107
        self.chan = np.abs(self.chan - F)
        arr, draws = self._arrivals(t, rng_step, arrivals)                         # 178-196 / 159-177
        for (i, _k) in draws:
            nxt[:, i, s.d[i] - 1] = arr[:, i]
            self.received[:, i] += arr[:, i]
        self.buffers = nxt
        obs, state = self._obs_state(chan_obs, ack)                                 # 199-209 / 180-186
        done = t >= s.episode_length                                                # 233-236
        return dict(obs=obs, state=state, rewards=rewards, done=done, ack=ack, success=success,
                    buffers=self.buffers.copy(), chan=self.chan.copy(), received=self.received.copy(),
                    discarded=self.discarded.copy(), sel_q=self.sel_q.copy(), sel_n=self.sel_n.copy(),
                    flips=F, arrivals=arr)

    def _step_single(self, actions, rng_step, flips, arrivals):
        """D2DEnv.step (env.py:116-213) for every env; self.timestep already incremented."""
        s = self.spec
        t = self.timestep
        E, N = self.E, s.N
        actions = np.asarray(actions).reshape(E, N)
        ack = np.zeros((E, 1))
        success = np.zeros((E, N), dtype=bool)
        nxt = self.buffers.copy()
        for e in range(E):
            has = (self.buffers[e].sum(1) > 0) * 1.                                 # 124
            att = (actions[e] != 0) * has                                           # 125
            n_att = att.sum()                                                       # 126
            if n_att == 1:                                                          # 129
                idx = int(att.nonzero()[0][0])
                decoded = self.chan[e, idx]   # binomial(1, channel_state[idx]), state in {0, 1} (101-103)
                if decoded:
                    a = 1                                                           # 136
                    self.successful_transmissions[e] += 1
                    col = nxt[e, idx].nonzero()[0]                                  # 141-142
                    nxt[e, idx, col.min()] -= 1
                    success[e, idx] = True
                else:
                    a = 0                                                           # 144-145
                    self.channel_errors[e] += 1
            elif n_att > 1:
                a = -1                                                              # 147-148
                self.n_collisions[e] += 1
            else:
                a = 0                                                               # 150
            ack[e, 0] = a
        expired = nxt[:, :, 0].copy()                                               # 109-113, 155-156
        nxt = np.concatenate([nxt[:, :, 1:], np.zeros((E, N, 1), dtype=np.int64)], axis=2)
        self.discarded += expired
        Fl = self._flips(rng_step, flips)                                           # 105-107, 157
        self.chan = np.where(Fl != 0, 1 - self.chan, self.chan)
        arr, draws = self._arrivals(t, rng_step, arrivals)                         # 160-181
        for (i, _k) in draws:
            nxt[:, i, s.d[i] - 1] = arr[:, i]
            self.received[:, i] += arr[:, i]
        self.buffers = nxt
        obs, state = self._obs_state(None, ack)                                     # 184-205
        done = t >= s.episode_length                                                # 223-226
        return dict(obs=obs, state=state, rewards=ack[:, 0].copy(), done=done, ack=ack, success=success,
                    buffers=self.buffers.copy(), chan=self.chan.copy(), received=self.received.copy(),
                    discarded=self.discarded.copy(), channel_errors=self.channel_errors.copy(),
                    n_collisions=self.n_collisions.copy(), flips=Fl, arrivals=arr)

    # -------------------------------------------------------------- metrics
    def compute_jains(self):
        out = np.zeros(self.E)
        for e in range(self.E):
            sc = np.array([1 - self.discarded[e, k] / self.received[e, k] if self.received[e, k] > 0 else 1
                           for k in range(self.spec.N)], dtype=np.float64)
            out[e] = sc.sum() ** 2 / self.spec.N / (sc ** 2).sum()
        return out

    def compute_urllc(self):
        return 1 - self.discarded.sum(1) / self.received.sum(1)

    def compute_channel_score(self):
        return np.where(self.sel_n != 0, self.sel_q / np.maximum(self.sel_n, 1), 1.0)
