"""D2DEnv — drop-in for /root/reference/envs/env.py (single shared channel).

Same constructor kwargs, attributes, spaces, reset()/step() structures and
metrics as the reference class (lines 4-250); every slot (attempt count,
decode, ACK, packet removal, expiry, per-agent channel flips, arrivals and
the neighbourhood obs/state emission) is one HIP kernel over `n_envs` envs
(csrc/env_kernels.hip single_kernel).  Extra kwargs: n_envs, device, seed
(see combinatorial_env.py).

Behavioural notes:
  * actions are 0/1 per agent (the Discrete(2) action space); the reference
    multiplies them by has_a_packet and sums, so only 0/1 keeps its count
    meaningful — other values raise here;
  * decode_signal draws Binomial(1, channel_state[idx]) but the state only
    ever takes the values 1 (reset, :78) and 1 - state (:105-107), so the
    decode is the attempter's channel bit; `channel_decoding` is stored and,
    as in the reference, unused (its use at :77 is commented out);
  * `channel_switch` may be a scalar or one probability per agent (it is
    the Binomial p of evolve_channel, :106).
"""
import numpy as np

from d2dhip.spec import EnvSpec

from . import spaces
from ._device_env import DeviceEnvBase


class D2DEnv(DeviceEnvBase):
    kind = "single"

    def __init__(self,
                 n_agents,
                 deadlines,
                 lbdas,
                 period=5,
                 arrival_probs=None,
                 offsets=None,
                 episode_length=100,
                 traffic_model='aperiodic',
                 periodic_devices=[],
                 reward_type=0,
                 channel_switch=0.2,
                 channel_decoding=0.8,
                 neighbourhoods=None,
                 verbose=False,
                 n_envs=1,
                 device=None,
                 seed=None):
        self.verbose = verbose
        self.n_agents = n_agents
        self.n_channels = 1
        self.lbdas = lbdas
        self.period = period
        self.deadlines = np.asarray(deadlines)
        self.arrival_probs = arrival_probs
        self.offsets = offsets
        self.episode_length = episode_length
        self.traffic_model = traffic_model
        self.reward_type = reward_type
        self.periodic_devices = periodic_devices
        pdev = set(int(i) for i in np.asarray(periodic_devices).reshape(-1)) if periodic_devices is not None else set()
        self.aperiodic_devices = [i for i in range(self.n_agents) if i not in pdev]
        self.channel_switch = channel_switch
        self.channel_decoding = channel_decoding
        if neighbourhoods is None:
            self.neighbourhoods = [[k] for k in range(self.n_agents)]
        else:
            self.neighbourhoods = neighbourhoods
        d = self.deadlines
        self.observation_space = spaces.Tuple([spaces.Box(low=-float('inf'), high=float('inf'),
                                                          shape=(int(d[list(nb)].sum()) + len(nb) + 1,))
                                               for nb in self.neighbourhoods])
        self.action_space = spaces.Tuple([spaces.Discrete(2) for _ in range(self.n_agents)])
        self.state_space = spaces.Box(low=-float('inf'), high=float('inf'), shape=(int(d.sum()) + self.n_agents + 1,))
        self._init_common(n_envs, device, seed)

    def _make_spec(self):
        return EnvSpec("single", self.n_agents, 1, self.deadlines, self.lbdas, self.period, self.arrival_probs,
                       self.offsets, self.episode_length, self.traffic_model, self.periodic_devices, False,
                       self.channel_switch, neighbourhoods=self.neighbourhoods)

    # device counters (env.py:144-150); reset() zeroes them in the kernel
    def _counter(self, t):
        if self._batch is None:
            return 0
        v = t.cpu().numpy().astype(np.int64)
        return int(v[0]) if self.n_envs == 1 else v

    @property
    def channel_errors(self):
        return self._counter(self._batch.sel_quality) if self._batch is not None else 0

    @channel_errors.setter
    def channel_errors(self, v):
        if np.any(np.asarray(v) != 0):
            raise AttributeError("channel_errors is the device counter; only reset() clears it")

    @property
    def n_collisions(self):
        return self._counter(self._batch.sel_count) if self._batch is not None else 0

    @n_collisions.setter
    def n_collisions(self, v):
        if np.any(np.asarray(v) != 0):
            raise AttributeError("n_collisions is the device counter; only reset() clears it")

    def decode_signal(self, attempts_idx):
        """API parity (env.py:101-103); the kernel decodes with the channel bit itself."""
        return np.random.binomial(1, self.channel_state[attempts_idx])

    def _pack_actions(self, actions):
        import torch
        a = np.asarray(actions).reshape(self.n_envs, self.n_agents)
        if a.size and not np.all((a == 0) | (a == 1)):
            raise ValueError("D2DEnv actions must be 0 or 1 per agent (Discrete(2))")
        return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint8)).to(self.batch().device)

    # ------------------------------------------------ reference numpy API
    def step(self, actions):
        s = self.spec
        b = self.batch()
        a = self._pack_actions(actions)
        out = b.step(a, want_obs=True, want_state=True, want_ack=True, want_success=True)
        self.timestep = b.timestep
        self.last_time_transmitted += 1
        self.last_attempts += 1
        ack = out["ack"].cpu().numpy().astype(np.float64)                       # [E]
        succ = out["success"].cpu().numpy().astype(bool)
        obs = out["obs"].cpu().numpy()
        state = out["state"].cpu().numpy()
        self.last_time_transmitted[succ.reshape(self.last_time_transmitted.shape)] = 1.0
        if self.n_envs == 1:
            self.successful_transmissions += int(ack[0] == 1)
            self.last_feedback = float(ack[0])
            rewards = np.zeros(s.N) + ack[0]                                      # env.py:207
        else:
            self.successful_transmissions = self.successful_transmissions + (ack == 1).astype(np.int64)
            self.last_feedback = ack
            rewards = np.zeros((self.n_envs, s.N)) + ack[:, None]
        if self.verbose:
            print(f"Timestep {self.timestep}")
            print(f"Channels {self.channel_state}")
            print(f"Channel errors: {self.channel_errors}")
            print(f"Reward {rewards}")
            print(f"Received packets {self.received_packets}")
            print(f"Number of discarded packets {self.discarded_packets.sum()}")
            print("")
        done = self.timestep >= s.episode_length
        return self._ref_obs(obs, None), self._ref_state(state, None, reset=False), rewards, done, {}

    def _ref_obs(self, obs, ack):
        s = self.spec
        out = []
        for k in range(s.N):
            o = obs[:, k, : s.obs_len[k]].astype(np.float64)
            out.append(o[0] if self.n_envs == 1 else o)
        return out

    def _ref_state(self, state, ack, reset):
        st = state[:, : self.spec.S].astype(np.float64)                          # one array (env.py:97-98, 204-205)
        return st[0] if self.n_envs == 1 else st

    def compute_channel_score(self):
        raise AttributeError("D2DEnv has no channel score (the reference class defines none)")
