"""Shared learner machinery: reference-compatible networks + agent-stacked
parameters so all N per-agent networks run as ONE batched GEMM chain.

Reference networks (/root/reference/algorithms/ippo.py:7-90, d2d_ppo.py:17-98):
  Policy  Linear(in,H) -> ReLU -> Linear(H,A) -> softmax      (orthogonal gain 2, zero bias)
  Value   Linear(in,H) -> ReLU -> Linear(H,1)
  RNN     GRU(in,H) over the window from h0=0 -> Linear(H,H) -> ReLU -> Linear(H,out)
          (orthogonal gain 3 on the Linears) -> softmax | sigmoid | none

Each agent still owns its nn.Module (same construction order, hence the same
torch-RNG-driven init as the reference under the same seed, and the same
state_dict keys for agent_{i}.pth), but after construction its parameters are
re-pointed to slices of agent-stacked tensors [N, ...].  The learners run the
stacked tensors through torch.bmm/baddbmm (hipBLASLt MFMA on MI355X), so a
forward/backward for all agents is a handful of launches instead of N x
batch-1 calls.  Agents with shorter observations (heterogeneous deadlines)
use a prefix of the input columns; the padded weight columns stay exactly
zero (zero inputs -> zero gradients -> zero Adam updates).
"""
import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.distributions import Bernoulli, Categorical


def init_weights(m, gain):
    if (type(m) == nn.Linear) | (type(m) == nn.Conv2d):
        nn.init.orthogonal_(m.weight, gain)
        if m.bias is not None:
            nn.init.zeros_(m.bias)


class RNN(torch.nn.Module):
    def __init__(self, n_inputs, n_outputs, hidden_size=100, combinatorial=False, use_activation=True, **kwargs):
        super().__init__()
        self.hidden_size = hidden_size
        self.combinatorial = combinatorial
        self.use_activation = use_activation
        self.lstm = nn.GRU(n_inputs, hidden_size, 1)
        self.layers = nn.Sequential(nn.Linear(hidden_size, hidden_size), nn.ReLU(), nn.Linear(hidden_size, n_outputs))
        self.layers.apply(lambda x: init_weights(x, 3))

    def init_hidden(self, batch_size):
        return (torch.zeros(1, batch_size, self.hidden_size), torch.zeros(1, batch_size, self.hidden_size))

    def forward(self, obs):
        if len(obs.shape) == 2:
            obs = obs.unsqueeze(0)
        w = self.lstm
        h = gru_window(obs.unsqueeze(0), w.weight_ih_l0.unsqueeze(0), w.weight_hh_l0.unsqueeze(0),
                       w.bias_ih_l0.unsqueeze(0), w.bias_hh_l0.unsqueeze(0))[0]
        out = self.layers(h)
        if self.use_activation:
            out = torch.sigmoid(out) if self.combinatorial else F.softmax(out, dim=1)
        return out


class Policy(nn.Module):
    def __init__(self, num_inputs, n_actions, hidden_size=100):
        super().__init__()
        self.n_actions = n_actions
        self.linear1 = nn.Linear(num_inputs, hidden_size)
        self.linear2 = nn.Linear(hidden_size, n_actions)
        init_weights(self.linear1, 2)
        init_weights(self.linear2, 2)

    def forward(self, inputs):
        x = inputs.unsqueeze(0) if len(inputs.shape) == 1 else inputs
        x = F.relu(self.linear1(x))
        return F.softmax(self.linear2(x), dim=1)


class Value(nn.Module):
    def __init__(self, num_inputs, hidden_size=100):
        super().__init__()
        self.linear1 = nn.Linear(num_inputs, hidden_size)
        self.linear2 = nn.Linear(hidden_size, 1)
        init_weights(self.linear1, 2)
        init_weights(self.linear2, 2)

    def forward(self, inputs):
        x = inputs.unsqueeze(0) if len(inputs.shape) == 1 else inputs
        return self.linear2(F.relu(self.linear1(x)))


# ----------------------------------------------------------------- GRU window
def gru_window(x, w_ih, w_hh, b_ih, b_hh):
    """Batched-over-agents GRU from h0 = 0 over a window.
    x [G][B][L][in], w_ih [G][3H][in], w_hh [G][3H][H], b_* [G][3H] -> last hidden [G][B][H].
    Gate order (r, z, n) and formula of torch.nn.GRU."""
    G, B, L, _ = x.shape
    H = w_hh.shape[2]
    gi = torch.baddbmm(b_ih.unsqueeze(1), x.reshape(G, B * L, -1), w_ih.transpose(1, 2)).view(G, B, L, 3 * H)
    h = None
    for t in range(L):
        g = gi[:, :, t]
        if h is None:
            gh = b_hh.unsqueeze(1).expand(G, B, 3 * H)
        else:
            gh = torch.baddbmm(b_hh.unsqueeze(1), h, w_hh.transpose(1, 2))
        r = torch.sigmoid(g[..., :H] + gh[..., :H])
        z = torch.sigmoid(g[..., H:2 * H] + gh[..., H:2 * H])
        n = torch.tanh(g[..., 2 * H:] + r * gh[..., 2 * H:])
        h = (1 - z) * n if h is None else (1 - z) * n + z * h
    return h


# ------------------------------------------------------------ stacked params
class StackedNets:
    """Agent-stacked copy of N per-agent modules (all Policy, all Value or all RNN).

    Parameters live in `self.params` (dict name -> nn.Parameter [N, ...]); each
    agent module's parameters become views into them."""

    def __init__(self, modules, in_dims, kind, device, act=None):
        self.kind = kind  # 'mlp' or 'rnn'
        self.N = len(modules)
        self.act = act    # 'softmax' | 'sigmoid' | None
        self.in_dims = [int(d) for d in in_dims]
        self.F = max(self.in_dims)
        m0 = modules[0]
        dev = torch.device(device)
        if kind == "mlp":
            H = m0.linear1.out_features
            A = m0.linear2.out_features
            shapes = {"w1": (H, self.F), "b1": (H,), "w2": (A, H), "b2": (A,)}
            srcs = lambda m: {"w1": m.linear1.weight, "b1": m.linear1.bias,  # noqa: E731
                              "w2": m.linear2.weight, "b2": m.linear2.bias}
        else:
            H = m0.hidden_size
            A = m0.layers[2].out_features
            shapes = {"w_ih": (3 * H, self.F), "w_hh": (3 * H, H), "b_ih": (3 * H,), "b_hh": (3 * H,),
                      "w1": (H, H), "b1": (H,), "w2": (A, H), "b2": (A,)}
            srcs = lambda m: {"w_ih": m.lstm.weight_ih_l0, "w_hh": m.lstm.weight_hh_l0,  # noqa: E731
                              "b_ih": m.lstm.bias_ih_l0, "b_hh": m.lstm.bias_hh_l0,
                              "w1": m.layers[0].weight, "b1": m.layers[0].bias,
                              "w2": m.layers[2].weight, "b2": m.layers[2].bias}
        self.H, self.A = H, A
        self.params = {}
        with torch.no_grad():
            for name, shp in shapes.items():
                # stacked where the modules live (host after construction), then ONE copy to the device
                # (per-agent copies were 2 x N x 4 hipMemcpy calls per network)
                t = torch.zeros((self.N,) + shp, dtype=torch.float32)
                for k, m in enumerate(modules):
                    src = srcs(m)[name].detach().to("cpu", torch.float32)
                    if name in ("w1", "w_ih") and not (kind == "rnn" and name == "w1"):
                        t[k, :, : self.in_dims[k]] = src
                    else:
                        t[k] = src
                self.params[name] = nn.Parameter(t.to(dev))
        for k, m in enumerate(modules):
            self._bind(m, k)

    def _bind(self, m, k):
        """Re-point module m's parameters to views of the stacked storage."""
        p = {n: t.data[k] for n, t in self.params.items()}
        d = self.in_dims[k]
        m.to(self.params["b1"].device)
        if self.kind == "mlp":
            m.linear1.weight = nn.Parameter(p["w1"][:, :d])
            m.linear1.bias = nn.Parameter(p["b1"])
            m.linear2.weight = nn.Parameter(p["w2"])
            m.linear2.bias = nn.Parameter(p["b2"])
        else:
            m.lstm.weight_ih_l0 = nn.Parameter(p["w_ih"][:, :d])
            m.lstm.weight_hh_l0 = nn.Parameter(p["w_hh"])
            m.lstm.bias_ih_l0 = nn.Parameter(p["b_ih"])
            m.lstm.bias_hh_l0 = nn.Parameter(p["b_hh"])
            m.layers[0].weight = nn.Parameter(p["w1"])
            m.layers[0].bias = nn.Parameter(p["b1"])
            m.layers[2].weight = nn.Parameter(p["w2"])
            m.layers[2].bias = nn.Parameter(p["b2"])

    def parameters(self):
        return list(self.params.values())

    def forward(self, x):
        """x: mlp [N][B][F]; rnn [N][B][L][F]  ->  [N][B][A] (activation applied)."""
        p = self.params
        if self.kind == "mlp":
            h = F.relu(torch.baddbmm(p["b1"].unsqueeze(1), x, p["w1"].transpose(1, 2)))
        else:
            h = gru_window(x, p["w_ih"], p["w_hh"], p["b_ih"], p["b_hh"])
            h = F.relu(torch.baddbmm(p["b1"].unsqueeze(1), h, p["w1"].transpose(1, 2)))
        out = torch.baddbmm(p["b2"].unsqueeze(1), h, p["w2"].transpose(1, 2))
        if self.act == "softmax":
            return F.softmax(out, dim=-1)
        if self.act == "sigmoid":
            return torch.sigmoid(out)
        return out

    def grad_norm_clip_(self, max_norm):
        """Per-agent torch.nn.utils.clip_grad_norm_(agent params, max_norm) (d2d_ppo.py:211)."""
        sq = None
        for t in self.params.values():
            if t.grad is None:
                continue
            s = t.grad.pow(2).reshape(self.N, -1).sum(1)
            sq = s if sq is None else sq + s
        if sq is None:
            return None
        norm = sq.sqrt()
        coef = (max_norm / (norm + 1e-6)).clamp(max=1.0)
        for t in self.params.values():
            if t.grad is not None:
                t.grad.mul_(coef.view((self.N,) + (1,) * (t.dim() - 1)))
        return norm


def make_dist(probs, combinatorial):
    if combinatorial:
        return Bernoulli(probs=probs, validate_args=False)
    return Categorical(probs=probs, validate_args=False)


def unpack_actions(masks, C):
    """uint8/int16/int32 channel masks [...] -> float 0/1 [..., C]."""
    bits = (masks.to(torch.int64).unsqueeze(-1) >> torch.arange(C, device=masks.device)) & 1
    return bits.to(torch.float32)


def rnn_windows(obs_seq, L, episode_length):
    """preprocess_input_for_rnn (ippo.py:390-403) on device for a batch of sequences.
    obs_seq [B][T][F] (T = whole rollout of one env, episodes of `episode_length`)
    -> [B][T][L][F], window i = obs[i-L+1 .. i] within the episode, front-zero-padded."""
    B, T, Fd = obs_seq.shape
    t = torch.arange(T, device=obs_seq.device)
    j = torch.arange(L, device=obs_seq.device)
    src = t.view(T, 1) - (L - 1) + j.view(1, L)                       # [T][L]
    ep_start = (t // episode_length) * episode_length
    valid = src >= ep_start.view(T, 1)
    idx = src.clamp(min=0)
    win = obs_seq[:, idx]                                              # [B][T][L][F]
    return win * valid.view(1, T, L, 1).to(obs_seq.dtype)


def as_numpy(x):
    return x.detach().cpu().numpy() if torch.is_tensor(x) else np.asarray(x)


def sqrt_safe(x):
    return math.sqrt(max(x, 0.0))
