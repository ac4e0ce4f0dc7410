"""CombinatorialEnv — drop-in for /root/reference/envs/combinatorial_env.py.

Same constructor kwargs, attributes, spaces, reset()/step() structures and
metrics as the reference class (lines 6-264); the slot itself (collision
detection, ACK, packet removal, expiry, Markov channel flips, arrivals,
obs/state emission) runs as one HIP kernel on the MI355X for all `n_envs`
envs.  Extra kwargs: n_envs (default 1), device (default current GPU), seed
(Philox key; default drawn from the global numpy RNG).

Behavioural notes: actions are binary masks (non-zero
= attempt); `periodic_devices` may be a list or an ndarray (the reference's
`!= []` check raises on an ndarray under NumPy 2).
"""
import numpy as np

from . import spaces
from ._device_env import DeviceEnvBase, make_spec


class CombinatorialEnv(DeviceEnvBase):
    kind = "comb"

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
                 collision_type="pessimistic",
                 homogeneous_size=False,
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
        self.collision_type = collision_type
        self.homogeneous_size = homogeneous_size
        self.reward_type = reward_type
        self.periodic_devices = periodic_devices
        pdev = set(int(i) for i in np.asarray(periodic_devices).reshape(-1)) if periodic_devices is not None else set()
        self.aperiodic_devices = [i for i in range(self.n_agents) if i not in pdev]
        if channel_switch is None:
            self.channel_switch = np.zeros((self.n_agents, self.n_channels))
        else:
            self.channel_switch = channel_switch
        D = int(self.deadlines.max())
        if not self.homogeneous_size:
            self.observation_space = spaces.Tuple([spaces.Box(low=-float('inf'), high=float('inf'),
                                                              shape=(int(self.deadlines[k]) + 2 * self.n_channels,))
                                                   for k in range(self.n_agents)])
        else:
            self.observation_space = spaces.Tuple([spaces.Box(low=-float('inf'), high=float('inf'),
                                                              shape=(D + 2 * self.n_channels,))
                                                   for _ in range(self.n_agents)])
        self.action_space = spaces.Tuple([spaces.MultiBinary(self.n_channels) for _ in range(self.n_agents)])
        self.state_space = spaces.Box(low=-float('inf'), high=float('inf'),
                                      shape=(int(self.deadlines.sum()) + self.n_channels * (self.n_agents + 1),))
        self.selected_channel_qualities = 0   # never incremented by this env (reference quirk)
        self.number_selected_channel = 0
        self._init_common(n_envs, device, seed)

    def _make_spec(self):
        return make_spec("comb", self)

    def _pack_actions(self, actions):
        import torch
        from d2dhip.envbatch import pack_masks
        a = np.asarray(actions)
        if self.n_envs == 1:
            a = a.reshape(1, self.n_agents, self.n_channels)
        else:
            a = a.reshape(self.n_envs, self.n_agents, self.n_channels)
        return torch.from_numpy(pack_masks(a, self.n_channels)).to(self.batch().device)
