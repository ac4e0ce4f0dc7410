"""Heuristic MAC baselines (reference: /root/reference/algorithms/baselines.py).

Same classes, constructor kwargs, `act()` semantics and `run()` return tuples:
  RandomAccess                  (baselines.py:5-45)    channel_selection_env, uniform channel id
  EarliestDeadlineFirstScheduler (:48-111)              D2DEnv, the agent with the earliest deadline
  GFAccess                      (:113-168)             D2DEnv, Bernoulli(p) attempts
  CombinatorialRandomAccess     (:171-222)             combinatorial_env, Bernoulli(p) per channel

`run()` with `n_envs == 1` is the reference's host loop (actions from the global numpy
stream, one env step per slot).  With `n_envs > 1` the episodes run E at a time on the
GPU: the policy is a device op on the env's own state (Philox for the random policies,
a byte-scan + argmin for EDF), the env kernel steps all E envs, and the episode metrics
are device reductions over the batch — the same statistics, E episodes per wave.

Reference defects fixed: EDF.run unpacks the D2DEnv state (one array)
into (buffers, channels) and GFAccess.run reads `buffer_state` before assigning it, so
neither runs in the reference; here both read the env's current buffers / channel states.
RandomAccess.act reshapes the concatenated buffers to (N, D_max), which only works for
equal deadlines; here each agent's deadline-length slice is summed.
"""
import math

import numpy as np


# ------------------------------------------------------------------ host loop (n_envs == 1)
def _episode_stats(env, rewards_episode):
    return (np.sum(rewards_episode), env.received_packets.sum(), env.discarded_packets.sum(), env.compute_jains())


def _summary(recv, disc, jains, extra, rewards, extra_kind):
    score = 1 - np.sum(disc) / np.sum(recv)
    ex = np.mean(extra) if extra_kind == "channel_score" else np.sum(extra)
    return score, np.mean(jains), ex, np.mean(rewards)


# ------------------------------------------------------------ device loop (n_envs > 1)
def _run_device(env, act, n_episodes, extra_kind):
    """E episodes per wave on the GPU.  act(b) -> action buffer [E][N] for the current slot."""
    import torch
    b = env.batch()
    s = b.spec
    E, L, N = b.E, env.episode_length, s.N
    waves = max(1, math.ceil(n_episodes / E))
    recv, disc, jains, extra, rewards = [], [], [], [], []
    acc = torch.zeros(E, dtype=torch.int64, device=b.device)
    for _ in range(waves):
        env.reset_batched(want_obs=False)
        acc.zero_()
        for _t in range(L):
            out = env.step_batched(act(b), want_obs=False)
            acc += out["reward"]
        r = b.received.double()
        d = b.discarded.double()
        u = torch.where(r > 0, 1 - d / r.clamp(min=1), torch.ones_like(r))
        recv.append(r.sum(1))
        disc.append(d.sum(1))
        jains.append(u.sum(1) ** 2 / N / (u ** 2).sum(1))
        if extra_kind == "channel_errors":
            extra.append(b.sel_quality.double() if s.kind == "single" else torch.zeros(E, dtype=torch.float64,
                                                                                       device=b.device))
        elif s.kind == "chsel":
            q, n = b.sel_quality.double(), b.sel_count.double()
            extra.append(torch.where(n != 0, q / n.clamp(min=1), torch.ones_like(q)))
        else:
            extra.append(torch.ones(E, dtype=torch.float64, device=b.device))  # comb counters stay 0
        rewards.append(acc.double() * N)   # np.sum over the broadcast per-agent reward vectors
    cat = lambda xs: torch.cat(xs)[:n_episodes].cpu().numpy()  # noqa: E731
    return _summary(cat(recv), cat(disc), cat(jains), cat(extra), cat(rewards), extra_kind)


def _has_packet(b):
    return (b.buffers != 0).any(-1)                                    # [E][N]


# ------------------------------------------------------------------------- baselines
class RandomAccess:
    """Uniform random channel id for agents with a packet (baselines.py:5-45)."""

    def __init__(self, env, verbose=False):
        self.env = env
        self.verbose = verbose

    def act(self, buffers):
        e = self.env
        offs = np.concatenate([[0], np.cumsum(e.deadlines)])
        n_packets = np.array([np.asarray(buffers)[offs[k]:offs[k + 1]].sum() for k in range(e.n_agents)])
        actions = np.random.choice(np.arange(0, e.n_channels + 1), size=e.n_agents)
        actions[n_packets == 0] = 0
        return actions

    def _act_device(self, b):
        a = b.sample_actions()                                         # uniform id in 0..C (Philox)
        return a * _has_packet(b).to(a.dtype)

    def run(self, n_episodes):
        env = self.env
        if env.n_envs > 1:
            out = _run_device(env, self._act_device, n_episodes, "channel_score")
        else:
            recv, disc, jains, score, rewards = [], [], [], [], []
            for _ in range(n_episodes):
                rewards_episode = []
                done = False
                _, (buffer_state, _channel_state) = env.reset()
                while not done:
                    action = self.act(buffer_state)
                    _, next_state, reward, done, _ = env.step(action)
                    buffer_state = next_state[0]
                    rewards_episode.append(reward)
                r, rc, dc, j = _episode_stats(env, rewards_episode)
                rewards.append(r), recv.append(rc), disc.append(dc), jains.append(j)
                score.append(env.compute_channel_score())
            out = _summary(recv, disc, jains, score, rewards, "channel_score")
        if self.verbose:
            print(f"Channel score: {out[2]}")
        return out


class EarliestDeadlineFirstScheduler:
    """One transmitter per slot: the agent whose oldest packet expires first (lowest index
    on ties); a uniformly random agent when nobody has a packet (baselines.py:48-111)."""

    def __init__(self, env, use_channel=False, verbose=False):
        self.env = env
        self.use_channel = use_channel
        self.verbose = verbose
        self.name = "EDF"

    def preprocess_state(self, state):
        output = []
        for row in state:
            packets = np.nonzero(row)[0]
            output.append(packets.min() if len(packets) > 0 else -1)
        return np.array(output)

    def act(self, buffers):
        agg_state = self.preprocess_state(buffers)
        n_packets = (agg_state >= 0).sum()
        if n_packets > 0:
            has_a_packet = (agg_state + 1).nonzero()[0]
            action_idx = has_a_packet[agg_state[has_a_packet].argmin()]
        else:
            action_idx = np.random.randint(self.env.n_agents)
        actions = np.zeros(self.env.n_agents)
        actions[action_idx] = 1.
        return actions

    def _act_device(self, b):
        import torch
        s = b.spec
        E, N = b.E, s.N
        cells = b.buffers.view(torch.uint8).view(E, N, -1)[:, :, : s.D]
        col = torch.arange(s.D, device=b.device, dtype=torch.int32)
        first = torch.where(cells != 0, col, torch.full_like(col, 255)).amin(-1)     # earliest column, 255 = none
        if self.use_channel:
            first = torch.where(b.channels != 0, first, torch.full_like(first, 255))  # bad channel: buffer hidden
        idx = first.argmin(-1)                                                          # first minimum (ties: lowest k)
        none = first.amin(-1) == 255
        idx = torch.where(none, torch.randint(N, (E,), device=b.device), idx)
        a = torch.zeros((E, N), dtype=torch.uint8, device=b.device)
        a.scatter_(1, idx[:, None], 1)
        return a

    def run(self, n_episodes):
        env = self.env
        if env.n_envs > 1:
            out = _run_device(env, self._act_device, n_episodes, "channel_errors")
        else:
            recv, disc, jains, losses, rewards = [], [], [], [], []
            for _ in range(n_episodes):
                rewards_episode = []
                done = False
                env.reset()
                while not done:
                    buffer_state = np.array(env.current_buffers)
                    if self.use_channel:
                        buffer_state[~(np.asarray(env.channel_state) > 0.5)] = 0
                    action = self.act(buffer_state)
                    _, _, reward, done, _ = env.step(action)
                    rewards_episode.append(reward)
                r, rc, dc, j = _episode_stats(env, rewards_episode)
                rewards.append(r), recv.append(rc), disc.append(dc), jains.append(j)
                losses.append(env.channel_errors)
            out = _summary(recv, disc, jains, losses, rewards, "channel_errors")
        if self.verbose:
            print(f"Number of channel_losses: {out[2]}")
        return out


class GFAccess:
    """Grant-free access: every agent with a packet transmits with probability p
    (baselines.py:113-168)."""

    def __init__(self, env, transmission_prob=0.5, transmission_prob_list=[0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9, 1],
                 use_channel=False, verbose=False):
        self.env = env
        self.transmission_prob = transmission_prob
        self.transmission_prob_list = transmission_prob_list
        self.use_channel = use_channel
        self.verbose = verbose

    def act(self, buffers):
        n_packets = np.asarray(buffers).sum(1)
        actions = np.random.binomial(1, p=self.transmission_prob, size=self.env.n_agents)
        actions[n_packets == 0] = 0
        return actions

    def _act_device(self, b):
        a = b.sample_actions(self.transmission_prob)                   # Bernoulli(p) per agent (Philox)
        keep = _has_packet(b)
        if self.use_channel:
            keep = keep & (b.channels != 0)
        return a * keep.to(a.dtype)

    def get_best_transmission_probs(self, n_episodes):
        cv = []
        for tp in self.transmission_prob_list:
            self.transmission_prob = tp
            score, _, _, _ = self.run(n_episodes)
            cv.append(np.mean(score))
        return cv

    def run(self, n_episodes):
        env = self.env
        if env.n_envs > 1:
            out = _run_device(env, self._act_device, n_episodes, "channel_errors")
        else:
            recv, disc, jains, losses, rewards = [], [], [], [], []
            for _ in range(n_episodes):
                rewards_episode = []
                done = False
                env.reset()
                while not done:
                    buffer_state = np.array(env.current_buffers)
                    if self.use_channel:
                        buffer_state[~(np.asarray(env.channel_state) > 0.5)] = 0
                    action = self.act(buffer_state)
                    _, _, reward, done, _ = env.step(action)
                    rewards_episode.append(reward)
                r, rc, dc, j = _episode_stats(env, rewards_episode)
                rewards.append(r), recv.append(rc), disc.append(dc), jains.append(j)
                losses.append(env.channel_errors)
            out = _summary(recv, disc, jains, losses, rewards, "channel_errors")
        if self.verbose:
            print(f"Number of channel_losses: {out[2]}")
        return out


class CombinatorialRandomAccess:
    """Every agent attempts every channel with probability p (baselines.py:171-222)."""

    def __init__(self, env, transmission_prob=0.5, transmission_prob_list=None, verbose=False):
        self.env = env
        self.transmission_prob = transmission_prob
        self.transmission_prob_list = np.arange(0, 1, 0.1) if transmission_prob_list is None else transmission_prob_list
        self.verbose = verbose

    def act(self, buffers):
        return np.random.binomial(1, self.transmission_prob, (self.env.n_agents, self.env.n_channels))

    def _act_device(self, b):
        return b.sample_actions(self.transmission_prob)                # Bernoulli(p) per (agent, channel) masks

    def get_best_transmission_probs(self, n_episodes):
        cv = []
        for tp in self.transmission_prob_list:
            self.transmission_prob = tp
            score, _, _, _ = self.run(n_episodes)
            cv.append(np.mean(score))
        return cv

    def run(self, n_episodes):
        env = self.env
        if env.n_envs > 1:
            out = _run_device(env, self._act_device, n_episodes, "channel_score")
        else:
            recv, disc, jains, score, rewards = [], [], [], [], []
            for _ in range(n_episodes):
                rewards_episode = []
                done = False
                _, state = env.reset()
                while not done:
                    action = self.act(state[0])
                    _, state, reward, done, _ = env.step(action)
                    rewards_episode.append(reward)
                r, rc, dc, j = _episode_stats(env, rewards_episode)
                rewards.append(r), recv.append(rc), disc.append(dc), jains.append(j)
                score.append(env.compute_channel_score())
            out = _summary(recv, disc, jains, score, rewards, "channel_score")
        if self.verbose:
            print(f"Channel score: {out[2]}")
        return out
