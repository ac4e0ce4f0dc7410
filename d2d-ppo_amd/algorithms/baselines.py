"""Heuristic MAC baselines — host-side policies driving the device envs through
the reference env API (reference: /root/reference/algorithms/baselines.py).

Only CombinatorialRandomAccess (slotted ALOHA over the channel matrix) is on a
caller's path: xp_n_agents.py:137-140 runs it.  RandomAccess covers the
channel-selection env.  They use the global numpy stream for their actions,
like the reference (baselines.py:11-13, 181-183).
"""
import numpy as np


def _run(env, act, n_episodes):
    number_of_discarded, number_of_received, rewards_list, jains_index, channel_score = [], [], [], [], []
    for _ in range(n_episodes):
        rewards_episode = []
        done = False
        _, state = env.reset()
        while not done:
            action = act(state[0])
            _, next_state, reward, done, _ = env.step(action)
            state = next_state
            rewards_episode.append(reward)
        rewards_list.append(np.sum(rewards_episode))
        number_of_received.append(env.received_packets.sum())
        number_of_discarded.append(env.discarded_packets.sum())
        jains_index.append(env.compute_jains())
        channel_score.append(env.compute_channel_score())
    return (1 - np.sum(number_of_discarded) / np.sum(number_of_received), np.mean(jains_index),
            np.mean(channel_score), np.mean(rewards_list))


class RandomAccess:
    """Uniform random channel id for agents with a packet (baselines.py:5-45)."""

    def __init__(self, env, verbose=False):
        self.env = env
        self.verbose = verbose

    def act(self, buffers):
        e = self.env
        # buffer_state is the concatenation of the agents' deadline-length buffers
        offs = np.concatenate([[0], np.cumsum(e.deadlines)])
        n_packets = np.array([buffers[offs[k]:offs[k + 1]].sum() for k in range(e.n_agents)])
        actions = np.random.choice(np.arange(0, e.n_channels + 1), size=e.n_agents)
        actions[n_packets == 0] = 0
        return actions

    def run(self, n_episodes):
        return _run(self.env, self.act, n_episodes)


class CombinatorialRandomAccess:
    """Every agent attempts every channel with probability p (baselines.py:171-222)."""

    def __init__(self, env, transmission_prob=0.5, transmission_prob_list=None, verbose=False):
        self.env = env
        self.transmission_prob = transmission_prob
        self.transmission_prob_list = np.arange(0, 1, 0.1) if transmission_prob_list is None else transmission_prob_list
        self.verbose = verbose

    def act(self, buffers):
        return np.random.binomial(1, self.transmission_prob, (self.env.n_agents, self.env.n_channels))

    def get_best_transmission_probs(self, n_episodes):
        cv = []
        for tp in self.transmission_prob_list:
            self.transmission_prob = tp
            score, _, _, _ = self.run(n_episodes)
            cv.append(np.mean(score))
        return cv

    def run(self, n_episodes):
        out = _run(self.env, self.act, n_episodes)
        if self.verbose:
            print(f"Channel score: {out[2]}")
        return out
