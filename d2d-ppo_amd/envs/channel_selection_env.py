"""ChannelSelectionEnv — drop-in for /root/reference/envs/channel_selection_env.py.

Same constructor kwargs, attributes, spaces, reset()/step() structures and
metrics as the reference class (lines 5-236); each slot is one HIP kernel
over `n_envs` envs.  Extra kwargs: n_envs, device, seed (see
combinatorial_env.py).

Actions are a length-N vector of channel ids 0..C (the env's documented
contract, channel_selection_env.py:117).  The reference learners hand it an
(N, 1) array, which the reference broadcasts to (N, N) and mis-counts
(SURVEY Q4); here any (N, 1) input is flattened to (N,).
"""
import numpy as np

from . import spaces
from ._device_env import DeviceEnvBase, make_spec


class ChannelSelectionEnv(DeviceEnvBase):
    kind = "chsel"

    def __init__(self,
                 n_agents,
                 n_channels,
                 deadlines,
                 lbdas,
                 period=5,
                 arrival_probs=None,
                 offsets=None,
                 episode_length=100,
                 traffic_model='aperiodic',
                 periodic_devices=[],
                 reward_type=0,
                 channel_switch=None,
                 verbose=False,
                 n_envs=1,
                 device=None,
                 seed=None):
        self.verbose = verbose
        self.n_agents = n_agents
        self.n_channels = n_channels
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
        if channel_switch is None:
            self.channel_switch = np.zeros(self.n_agents)
        else:
            self.channel_switch = channel_switch
        self.observation_space = spaces.Tuple([spaces.Box(low=-float('inf'), high=float('inf'),
                                                          shape=(int(self.deadlines[k]) + self.n_channels + 1,))
                                               for k in range(self.n_agents)])
        self.action_space = spaces.Tuple([spaces.Discrete(self.n_channels + 1) for _ in range(self.n_agents)])
        self.state_space = spaces.Box(low=-float('inf'), high=float('inf'),
                                      shape=(int(self.deadlines.sum()) + self.n_channels + 1,))
        self._init_common(n_envs, device, seed)

    def _make_spec(self):
        return make_spec("chsel", self)

    @property
    def selected_channel_qualities(self):
        if self._batch is None:
            return 0
        v = self._batch.sel_quality.cpu().numpy().astype(np.int64)
        return int(v[0]) if self.n_envs == 1 else v

    @property
    def number_selected_channel(self):
        if self._batch is None:
            return 0
        v = self._batch.sel_count.cpu().numpy().astype(np.int64)
        return int(v[0]) if self.n_envs == 1 else v

    def decode_signal(self, attempts_idx):
        """Unused by the reference's step; kept for API parity (channel_selection_env.py:100-102)."""
        return np.random.binomial(1, self.channel_state[attempts_idx])

    def _pack_actions(self, actions):
        import torch
        a = np.asarray(actions).reshape(self.n_envs, self.n_agents)
        if a.size and (a.min() < 0 or a.max() > self.n_channels):
            raise ValueError(f"channel ids must be in [0, {self.n_channels}]")
        return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint8)).to(self.batch().device)
