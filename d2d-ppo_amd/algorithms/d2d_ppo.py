"""D2D-PPO — drop-in for /root/reference/algorithms/d2d_ppo.py (HAPPO-style:
per-agent actors, one centralized critic on the global state at the BS,
random agent permutation per epoch, compound ratio M passed agent to agent).

The sequential chain (d2d_ppo.py:429-436) feeds agent sigma_j the advantage
times the ratios of the agents before it, each computed from that agent's
parameters BEFORE its own optimizer step — and no agent's parameters change
until its own turn.  So M_{sigma_j} = A * r_{sigma_0} * ... * r_{sigma_{j-1}}
with every r from the epoch-start parameters: an exclusive prefix product
along the permutation.  All N actor updates of an epoch therefore
run as ONE agent-stacked forward/backward; the prefix is N elementwise
multiplies over [B] in sigma order, left to right exactly like the
reference's loop.  Per-agent clip_grad_norm_(20) and Adam are kept.
"""
import os

import numpy as np
import torch
import torch.nn.functional as F

from ._core import Policy, RNN, StackedNets, Value, init_weights, make_dist  # noqa: F401
from ._learner import BatchedLearnerBase
from .ippo import compute_gae, discount_rewards  # noqa: F401  (identical in both reference modules)


class PPO:
    """Per-agent actor (d2d_ppo.py:128-216)."""

    def __init__(self, num_inputs, n_actions, hidden_size=128, gamma=0.99, policy_lr=1e-3, beta_entropy=0.01,
                 useRNN=False, combinatorial=False, device='cpu', history_len=5, early_stopping=True):
        self.history_len = history_len
        self.useRNN = useRNN
        self.combinatorial = combinatorial
        self.early_stopping = early_stopping
        self.device = torch.device(device)
        self.n_actions = n_actions
        self.beta_entropy = beta_entropy
        if not self.useRNN:
            self.policy_network = Policy(num_inputs, n_actions, hidden_size)
        else:
            self.policy_network = RNN(num_inputs, n_actions, hidden_size, combinatorial=combinatorial)
        self.gamma = gamma
        self.policy_lr = policy_lr
        self.policy_optimizer = None

    def select_action(self, state, train=True):
        probs = self.policy_network(state.to(self.device))
        dist = make_dist(probs, self.combinatorial)
        if self.combinatorial:
            action = dist.sample().squeeze() if train else (dist.probs.squeeze() > 0.5) * 1.
            return action.cpu().detach().numpy(), dist.log_prob(action).mean(-1), dist.entropy().mean(-1)
        action = dist.sample() if train else probs.argmax(dim=1)
        return action.cpu().detach().numpy(), dist.log_prob(action), dist.entropy()

    def evaluate(self, states, actions):
        probs = self.policy_network(states.to(self.device).squeeze())
        dist = make_dist(probs, self.combinatorial)
        a = torch.as_tensor(actions).to(self.device)
        if self.combinatorial:
            return dist.log_prob(a).mean(-1), dist.entropy().mean(-1)
        return dist.log_prob(a), dist.entropy()

    def train_step(self, states, actions, log_probs_old, M, cliprange=0.1):
        if self.policy_optimizer is None:
            self.policy_optimizer = torch.optim.Adam(self.policy_network.parameters(), lr=self.policy_lr)
        M = M.to(self.device)
        log_probs, entropy = self.evaluate(states, actions)
        entropy = entropy.mean()
        ratio = torch.exp(log_probs - log_probs_old.to(self.device))
        policy_loss = -torch.min(ratio * M, torch.clamp(ratio, 1.0 - cliprange, 1.0 + cliprange) * M).mean() \
            - self.beta_entropy * entropy
        self.policy_optimizer.zero_grad()
        policy_loss.backward()
        torch.nn.utils.clip_grad_norm_(self.policy_network.parameters(), 20)
        self.policy_optimizer.step()
        return policy_loss.item(), ratio * M


def happo_chain(adv, ratio, perm):
    """M for every agent: adv [B], ratio [N][B] (detached), perm = sigma (np array of agent ids).
    M[sigma_j] = (((adv * r_sigma0) * r_sigma1) ... * r_sigma_{j-1}), multiplied left to right in
    float32 exactly like the reference's loop (torch.cumprod may accumulate in double on CPU)."""
    N = ratio.shape[0]
    perm = [int(i) for i in np.asarray(perm)]
    M = torch.empty_like(ratio)
    cur = adv
    for j, i in enumerate(perm):
        M[i] = cur
        if j + 1 < N:
            cur = ratio[i] * cur
    return M


class D2DPPO(BatchedLearnerBase):
    def __init__(self,
                 env,
                 hidden_size=128,
                 gamma=0.99,
                 policy_lr=1e-3,
                 value_lr=1e-3,
                 beta_entropy=0.01,
                 device=None,
                 useRNN=False,
                 save_path=None,
                 combinatorial=False,
                 history_len=10,
                 early_stopping=True):
        self.env = env
        self.history_len = history_len
        self.n_agents = env.n_agents
        self.hidden_size = hidden_size
        self.gamma = gamma
        self.policy_lr = policy_lr,   # tuples, as in the reference (d2d_ppo.py:239-240)
        self.value_lr = value_lr,
        self.beta_entropy = beta_entropy
        self.early_stopping = early_stopping
        self.useRNN = useRNN
        self.save_path = save_path
        self.combinatorial = combinatorial
        self.device = self._resolve_device(device)
        if self.device.type != "cuda":
            import d2dhip
            d2dhip.require_gpu()
        self.agents = [PPO(num_inputs=self.env.observation_space[k].shape[0],
                           n_actions=self.env.action_space[k].n,
                           hidden_size=hidden_size,
                           gamma=gamma,
                           policy_lr=policy_lr,
                           beta_entropy=beta_entropy,
                           useRNN=useRNN,
                           combinatorial=combinatorial,
                           history_len=history_len,
                           device=self.device,
                           early_stopping=early_stopping) for k in range(self.n_agents)]
        # The value network is at the BS (d2d_ppo.py:264-267)
        self.value_network = Value(self.env.state_space.shape[0], hidden_size)
        self.value_network = self.value_network.to(self.device)
        self.value_optimizer = torch.optim.Adam(self.value_network.parameters(), lr=value_lr)
        in_dims = [env.observation_space[k].shape[0] for k in range(self.n_agents)]
        self.policy = StackedNets([a.policy_network for a in self.agents], in_dims,
                                  "rnn" if useRNN else "mlp", self.device, act=self._policy_act())
        self.policy_optimizer = torch.optim.Adam(self.policy.parameters(), lr=policy_lr)
        self._setup_data_parallel(self.policy.parameters() + list(self.value_network.parameters()))

    # ------------------------------------------------------------ rollouts
    # round 5: the combinatorial env writes the rollout states as the central critic's bf16 operand (exact
    # integers; d2d_env_out.state_bf16) when the fused critic takes them -- no fp32 state buffer, no conversion
    # pass; D2D_STATE_BF16=0 keeps the fp32 buffer + d2d_states_to_bf16_padded (A/B)
    state_bf16_rollout = os.environ.get("D2D_STATE_BF16", "1") != "0"

    def _state_mode(self):
        H = self.value_network.linear1.weight.shape[0]
        bf = (self.state_bf16_rollout and self.kind == "comb" and bool(self.combinatorial) and self.critic_split
              and self.critic_fused and H % 4 == 0 and H <= 128)
        return "bf16" if bf else True

    def _rollout(self, num_episodes, teacher=None):
        ro = self._collect(num_episodes, train=True, want_state=self._state_mode(), teacher=teacher)
        self._phase("rollout")
        # the actor parameters the rollout sampled with (a device copy: 2.5 K floats per MLP agent), so the
        # first update epoch can prove they are unchanged (any in-place write: Adam, load(), a direct
        # load_state_dict on an agent's module, a broadcast) before taking the ratio = 1 shortcut
        ro.policy_snapshot = [p.detach().clone() for p in self.policy.parameters()]
        S = self.env.state_space.shape[0]
        ro.state_dim = S  # ro.state_seq: the env-major [E*T][S] fp32 states, materialised on first use
        # returns = discount_rewards(rewards (T,N)).mean(1) (d2d_ppo.py:333,339): every agent has the
        # same reward, so all N normalised columns are identical and their mean is that column
        zero_v = torch.zeros((ro.T, ro.E, 1), dtype=torch.float32, device=self.device)
        _, ret = self._gae(ro.rewards, zero_v, ro.dones, normalize_adv=False, normalize_ret=True)
        ro.ret_mean = ret[:, :, 0].t().reshape(-1)                                     # [E*T]
        self._phase("gae")
        return ro

    def create_rollouts(self, num_episodes=4):
        """Reference return structure (d2d_ppo.py:339): obs list, states (T,S), actions, log_probs (T,N),
        rewards.mean(1), returns.mean(1), scores, dones (env-major sample axis when n_envs > 1)."""
        ro = self._rollout(num_episodes)
        s = self.env.batch().spec
        N = s.N
        obs = ro.obs_f32.permute(2, 1, 0, 3).reshape(N, ro.E * ro.T, -1)
        obs_list = [obs[k, :, : s.obs_len[k]] for k in range(N)]
        acts = ro.actions.permute(1, 0, 2).reshape(ro.E * ro.T, N)
        if self.kind == "comb":
            from ._core import unpack_actions
            acts = unpack_actions(acts, s.C)
        rewards = ro.rewards.t().reshape(-1).double().cpu().numpy()
        dones = [bool(d) for d in ro.dones.cpu().tolist()] * ro.E
        return (obs_list, ro.state_seq, acts.cpu().numpy(), self._seq(ro.logp).t().cpu(), rewards,
                ro.ret_mean.cpu(), ro.scores, dones)

    # -------------------------------------------------------------- update
    def _epoch(self, ro, x, acts, logp_old, cliprange=0.1):
        """One reference epoch (d2d_ppo.py:413-448) for all agents at once."""
        # 1) Sample a cycle of agents — the global numpy stream, exactly like the reference
        cycle = np.arange(self.n_agents)
        np.random.shuffle(cycle)
        cycle = self._sync_perm(cycle)
        # 2) global advantage at the BS
        values = self.value_network(ro.state_seq).squeeze()
        v_te = values.detach().view(ro.E, ro.T).t().unsqueeze(2).contiguous()
        adv, _ = self._gae(ro.rewards, v_te, ro.dones, normalize_adv=True, normalize_ret=False)
        A = adv[:, :, 0].t().reshape(-1)                                                # [E*T]
        # 3) the agents' chain as one batched update
        log_probs, entropy = self._evaluate(x, acts)
        ratio = torch.exp(log_probs - logp_old)                                          # [N][B]
        M = happo_chain(A, ratio.detach(), cycle)
        surr1 = ratio * M
        surr2 = torch.clamp(ratio, 1.0 - cliprange, 1.0 + cliprange) * M
        ploss = -torch.min(surr1, surr2).mean(1) - self.beta_entropy * entropy.mean(1)    # [N]
        self.policy_optimizer.zero_grad()
        ploss.sum().backward()
        self._reduce_grads(self.policy.parameters())
        self.policy.grad_norm_clip_(20)
        self.policy_optimizer.step()
        # 4) critic update (d2d_ppo.py:440-446)
        value_loss = F.mse_loss(values, ro.ret_mean, reduction='mean')
        self.value_optimizer.zero_grad()
        value_loss.backward()
        self._reduce_grads(list(self.value_network.parameters()))
        torch.nn.utils.clip_grad_norm_(self.value_network.parameters(), 20)
        self.value_optimizer.step()
        pl = ploss.detach().cpu().numpy()
        return [float(pl[i]) for i in cycle], value_loss.detach()

    def _epoch_fused(self, ro, cliprange=0.1):
        """The same epoch with the actors on the HIP kernels: epoch-start ratios of every agent
        from the policy kernel (forced actions), the chain M, then the fused actor-gradient
        kernel with W = M and beta_entropy; clipping, Adam and the central critic in torch.
        Sample order here is time-major (t * E + e); the sums do not depend on it."""
        from d2dhip.update import actor_grads
        cycle = np.arange(self.n_agents)
        np.random.shuffle(cycle)
        cycle = self._sync_perm(cycle)
        crit = self._critic_split_forward(ro)
        values = crit[0] if crit is not None else self.value_network(ro.state_seq).squeeze()
        self._phase("critic_fwd")
        v_te = values.detach().view(ro.E, ro.T).t().unsqueeze(2).contiguous()
        adv, _ = self._gae(ro.rewards, v_te, ro.dones, normalize_adv=True, normalize_ret=False)
        self._phase("gae")
        T, E, N = ro.T, ro.E, self.n_agents
        A = adv[:, :, 0].reshape(-1)                                                   # [T*E]
        with torch.no_grad():
            if not self.useRNN and self._actors_unchanged_since(ro):
                # first epoch on this rollout: the epoch-start actors ARE the rollout's, and the
                # policy kernel's forced log-probs equal the sampled ones bit for bit, so every
                # ratio is exactly 1 and the chain is A for every agent (no forced pass needed).
                # Not for GRU policies: their training windows are padded, the rollout's were not (Q5)
                M = A.expand(N, T * E)
            else:
                M = self._chain_dev(A, self._logp_forced(ro), ro.logp, cycle, T, E)     # [N][T*E]
        self._phase("chain")
        pp = self.policy.params
        kind = "comb" if self.combinatorial else "chsel"
        beta = float(self.beta_entropy)
        if self.useRNN:  # GRU policies: BPTT over the padded training windows (gru_kernels.hip)
            from d2dhip import gru
            _, sa = gru.grads({k: v.data for k, v in pp.items()}, ro.obs, self._gru_kind(), self.history_len, ro.L,
                              M.view(N, T, E).permute(1, 2, 0), actions=ro.actions,
                              logp_old=ro.logp.permute(0, 2, 1), clip=cliprange, beta=beta,
                              grads=self._grad_buffers(pp))
        else:
            _, sa = actor_grads({k: v.data for k, v in pp.items()}, ro.obs, ro.actions, ro.logp.permute(0, 2, 1),
                                M.view(N, T, E).permute(1, 2, 0), kind, clip=cliprange, beta=beta,
                                grads=self._grad_buffers(pp))
        self._phase("actor_grad")
        self._reduce_grads(self.policy.parameters())
        self._phase("allreduce")
        self.policy.grad_norm_clip_(20)
        self.policy_optimizer.step()
        self._phase("adam")
        ploss = -(sa[:, 0] + beta * sa[:, 1]) / (T * E)
        if crit is not None:
            value_loss = self._critic_split_backward(ro, crit)
        else:
            value_loss = F.mse_loss(values, ro.ret_mean, reduction='mean')
            self.value_optimizer.zero_grad()
            value_loss.backward()
        self._phase("critic_grad")
        self._reduce_grads(list(self.value_network.parameters()))
        self._phase("allreduce")
        torch.nn.utils.clip_grad_norm_(self.value_network.parameters(), 20)
        self.value_optimizer.step()
        self._phase("adam")
        pl = ploss.detach().cpu().numpy()
        return [float(pl[i]) for i in cycle], value_loss.detach()

    def _actors_unchanged_since(self, ro):
        snap = getattr(ro, "policy_snapshot", None)
        if snap is None:
            return False
        return all(torch.equal(a, p.detach()) for a, p in zip(snap, self.policy.parameters()))

    # ------------------------------------------------ central critic on bf16 split GEMMs
    critic_split = True
    # every state width: at configs[1]'s S = 117 and configs[4]'s 8 / 16 agents (S = 128 / 248) the fp32
    # path's dW1 (K = the whole 819 K-sample batch, one output tile row) took 12.4-13.3 ms per 5-epoch
    # iteration against 2.3-2.6 ms for the split-K bf16 path (profiles/r04/critic_small.log)
    CRITIC_SPLIT_MIN_DIM = 0
    CRITIC_F32_FWD_MAX_DIM = 768  # below this state width the forward's first layer is one fp32 GEMM
    # round 5: the forward and the backward's per-sample glue as one HIP kernel over the bf16 operand
    # (csrc/critic_kernels.hip, d2d_central_critic_fwd; hidden a multiple of 4 up to 128); D2D_CRITIC_FUSED=0
    # keeps the hipBLASLt forward GEMM + the dpre split kernel (A/B, tests)
    critic_fused = os.environ.get("D2D_CRITIC_FUSED", "1") != "0"

    def _critic_split_forward(self, ro):
        """Value(state) = linear2(relu(linear1(state))) (d2d_ppo.py:95-98) for all T*E states.  At
        S >= CRITIC_F32_FWD_MAX_DIM the first layer is ONE bf16 GEMM with fp32 output: the states are small
        integers (buffer counts, channel bits, ACKs) and so exact in bf16, and W1 is split three ways (h + m + l,
        exact), so the product is fp32-accurate at the bf16 matrix rate; below it the first layer is one fp32
        addmm on the fp32 states (the backward uses the bf16 operand either way).  Returns (values [B],
        pre-activation [H][B], hidden [H][B]) or None when the torch path applies (split off, S below
        CRITIC_SPLIT_MIN_DIM, or states that are not bf16-exact)."""
        S = ro.state_dim if "state_dim" in ro.__dict__ else ro.state_seq.shape[1]
        if not self.critic_split or S < self.CRITIC_SPLIT_MIN_DIM:
            return None
        xb = getattr(ro, "state_bf16", None)
        if xb is None:
            # the env kernels' states are small integers by construction (buffer counts <= 255, channel
            # bits, ACKs in {-1, 0, 1}), hence exact in bf16; the whole conversion is verified (row chunks,
            # so the check needs no second full-size fp32 copy) and a state that is not bf16-exact keeps
            # the critic on the torch fp32 GEMMs
            # one HIP pass converts and checks (d2d_f32_to_bf16_exact; was torch's conversion plus a
            # chunked compare / all() over a second fp32 copy: ~200 small launches per rollout at 256 agents)
            from d2dhip import _lib
            lib = _lib.require_gpu()
            st = ro.__dict__.get("states")
            if "state_seq" not in ro.__dict__ and st is not None and st.is_contiguous() and st.dim() == 3:
                # straight from the slot-major rollout buffer [T][E][stride] (no env-major fp32 copy), rows
                # padded with zero columns to a multiple of 8 (16-byte aligned GEMM rows: configs[1]'s S = 117)
                T_, E_ = st.shape[0], st.shape[1]
                S8 = -(-S // 8) * 8
                xb = torch.empty((E_ * T_, S8), dtype=torch.bfloat16, device=st.device)
                flag = torch.empty(1, dtype=torch.int32, device=st.device)
                _lib.check(lib.d2d_states_to_bf16_padded(T_, E_, S, st.shape[2], st.data_ptr(), xb.data_ptr(), S8,
                                                         flag.data_ptr(), _lib.stream_ptr()), "d2d_states_to_bf16_padded")
            else:
                # the env-major fp32 copy exists (a consumer asked for it): the same padded operand from it (as one
                # "slot" of B rows)
                sq = ro.state_seq.contiguous()
                S8 = -(-S // 8) * 8
                xb = torch.empty((sq.shape[0], S8), dtype=torch.bfloat16, device=sq.device)
                flag = torch.empty(1, dtype=torch.int32, device=sq.device)
                _lib.check(lib.d2d_states_to_bf16_padded(1, sq.shape[0], S, sq.shape[1], sq.data_ptr(), xb.data_ptr(), S8,
                                                         flag.data_ptr(), _lib.stream_ptr()), "d2d_states_to_bf16_padded")
            if int(flag.item()) != 0:
                self.critic_split = False  # fractional / large states: keep torch fp32
                return None
            ro.state_bf16 = xb
        l1, l2 = self.value_network.linear1, self.value_network.linear2
        H = l1.weight.shape[0]
        if self.critic_fused and H % 4 == 0 and H <= 128:
            return self._critic_fused_forward(ro, xb, S)
        if S < self.CRITIC_F32_FWD_MAX_DIM:
            # narrow states: the first layer as one fp32 GEMM on the env-major fp32 states (4 S + 4 H bytes
            # per sample) beats the split GEMM's [3H][B] fp32 output and its sum (2 S + 28 H bytes) below
            # S = 12 H; the backward still runs on the bf16 operand (split-K dW1).  c2 (S = 117): critic
            # forward 4.7 -> 2.8 ms per 5-epoch iteration (profiles/r04/critic_small*.log)
            with torch.no_grad():
                pre = torch.addmm(l1.bias[:, None], l1.weight, ro.state_seq.t())               # [H][B]
                hid = torch.relu(pre)
                v = torch.addmm(l2.bias[:, None], l2.weight, hid)[0]                           # [B]
            return v, pre, hid
        with torch.no_grad():
            w = l1.weight
            if xb.shape[1] > S:  # the operand's zero pad columns
                w = torch.nn.functional.pad(w, (0, xb.shape[1] - S))
            wh = w.to(torch.bfloat16)
            r = w - wh.float()
            wm = r.to(torch.bfloat16)
            wl = (r - wm.float()).to(torch.bfloat16)
            # computed transposed ([3H] x B): with H = 64 (the drivers' hidden size) the 3H = 192 output
            # rows are one GEMM tile, so the [B][S] states are streamed once (as [B][3H] the 192 columns
            # took two 128-wide tiles and read the states twice); larger H takes more row tiles either way
            z3 = torch.mm(torch.cat([wh, wm, wl], 0), xb.t(), out_dtype=torch.float32)   # [3H][B]
            pre = (z3[:H] + z3[H:2 * H]) + z3[2 * H:] + l1.bias[:, None]                # [H][B]
            hid = torch.relu(pre)
            v = torch.addmm(l2.bias[:, None], l2.weight, hid)[0]                           # [B]
        return v, pre, hid

    def _critic_fused_forward(self, ro, xb, S):
        """d2d_central_critic_fwd: V(state) of every sample and, against the critic target returns.mean
        (d2d_ppo.py:339, 440-446), dPre's three RNE bf16 parts [B][3H] and the sums db1 / dW2 / db2 / sum (v - R)^2
        per workgroup, in one pass over the bf16 operand (the critic's weights are the same at the backward).
        Returns (values [B], None, None, dhm, partial)."""
        from d2dhip import _lib
        lib = _lib.require_gpu()
        l1, l2 = self.value_network.linear1, self.value_network.linear2
        H = l1.weight.shape[0]
        B = xb.shape[0]
        dev = xb.device
        G = int(lib.d2d_central_critic_blocks(H, B))
        nimg = int(lib.d2d_central_critic_image_bytes(H, S))
        img = getattr(self, "_critic_img", None)
        if img is None or img.numel() < nimg // 16 or img.device != dev:
            img = self._critic_img = torch.empty((nimg // 16, 4), dtype=torch.int32, device=dev)  # 16-byte entries
        v = torch.empty(B, dtype=torch.float32, device=dev)
        dhm = torch.empty((B, 3 * H), dtype=torch.bfloat16, device=dev)
        part = torch.empty((max(G, 1), 2 * H + 2), dtype=torch.float32, device=dev)
        w1 = l1.weight.detach().contiguous()
        ret = ro.ret_mean.contiguous()
        _lib.check(lib.d2d_central_critic_fwd(H, B, S, xb.shape[1], xb.data_ptr(), w1.data_ptr(),
                                              l1.bias.detach().data_ptr(), l2.weight.detach().data_ptr(),
                                              l2.bias.detach().data_ptr(), ret.data_ptr(), img.data_ptr(), v.data_ptr(),
                                              dhm.data_ptr(), part.data_ptr(), G, _lib.stream_ptr()),
                   "d2d_central_critic_fwd")
        return v, None, None, dhm, part

    def _critic_split_backward(self, ro, crit):
        """Gradients of mse(V, returns) into the critic's .grad (what value_loss.backward() leaves,
        d2d_ppo.py:208-216): dW1 = dPreᵀ X on a three-way RNE bf16 split of dPre (~2^-24 relative per
        product term, torch fp32's level) against the exact bf16 states; dPre's split and the db1 / dW2 sums
        come from one HIP pass (d2d_critic_dpre_split3), dW1 from a split-K batched GEMM."""
        l1, l2 = self.value_network.linear1, self.value_network.linear2
        H = l1.weight.shape[0]
        if len(crit) == 5:  # the fused kernel already made dPre's parts and the sums
            v, _, _, dhm, part = crit
            with torch.no_grad():
                sums = part.sum(0)                                                      # db1 | dW2 | db2 | sum d^2
                value_loss = sums[2 * H + 1] / v.numel()
                if self.critic_dw1_hip:
                    gw1 = self._dw1_hip(dhm, ro.state_bf16, H, l1.weight.shape[1])              # [H][S]
                else:
                    g = self._dw1_gemm_bm(dhm, ro.state_bf16)[:, :l1.weight.shape[1]]   # [3H][S]
                    gw1 = (g[2 * H:] + g[H:2 * H]) + g[:H]
                grads = {l1.weight: gw1, l1.bias: sums[:H], l2.weight: sums[H:2 * H],
                         l2.bias: sums[2 * H:2 * H + 1]}
                for prm, gr in grads.items():
                    prm.grad = gr.reshape(prm.shape).contiguous()
            return value_loss
        v, pre, _ = crit
        with torch.no_grad():
            d = v - ro.ret_mean
            value_loss = (d * d).mean()
            dv = d * (2.0 / d.numel())                                                  # [B]
            g_b2 = dv.sum().reshape(1)
            # dpre = [pre > 0] w2^T dv as its RNE bf16 split parts [pH][B], db1 = sum_b dpre and
            # dW2 = sum_b relu(pre) dv, in one HIP pass over pre
            from d2dhip import _lib
            lib = _lib.require_gpu()
            B = pre.shape[1]
            G = int(lib.d2d_critic_dpre_blocks(B))
            pre_c, w2v, dv_c = pre.contiguous(), l2.weight.detach().reshape(-1).contiguous(), dv.contiguous()
            # dPre on a three-way RNE split (ABI v10): the two-way split's 2^-17 per product let near-zero dW1
            # elements take the other sign than fp32 autograd's, which Adam's first step turns into 2 lr moves
            # (the hidden-128 D2D reference trace's epoch-2 value loss, learner_d2d_mlp_comb_h128)
            dhm = torch.empty((3 * H, B), dtype=torch.bfloat16, device=pre.device)
            part = torch.empty((G, 2 * H), dtype=torch.float32, device=pre.device)
            _lib.check(lib.d2d_critic_dpre_split3(H, B, pre_c.data_ptr(), w2v.data_ptr(), dv_c.data_ptr(), dhm.data_ptr(),
                                                  part.data_ptr(), G, _lib.stream_ptr()), "d2d_critic_dpre_split3")
            sums = part.sum(0)                                                              # [2H]: db1 | dW2
            g = self._dw1_gemm(dhm, ro.state_bf16)[:, :l1.weight.shape[1]]                 # [3H][S]
            grads = {l1.weight: (g[2 * H:] + g[H:2 * H]) + g[:H], l1.bias: sums[:H], l2.weight: sums[H:],
                     l2.bias: g_b2}
            for prm, gr in grads.items():
                prm.grad = gr.reshape(prm.shape).contiguous()
        return value_loss

    # round 6: dW1 from the fused forward's dhm on the hand-written bf16 MFMA kernel (d2d_central_critic_dw1: the three
    # parts accumulated in one accumulator, no [3H][S] partial products, no hipBLASLt); D2D_CRITIC_DW1_HIP=0 keeps the
    # split-K bmm (A/B)
    critic_dw1_hip = os.environ.get("D2D_CRITIC_DW1_HIP", "1") != "0"

    def _dw1_hip(self, dhm, xb, H, S):
        """dW1 = sum_b dpre_b x_b^T [H][S] fp32 from dpre's parts dhm [B][3H] and the bf16 operand xb [B][ldx]."""
        from d2dhip import _lib
        lib = _lib.require_gpu()
        B, ldx = xb.shape[0], xb.shape[1]
        n = int(lib.d2d_central_critic_dw1_workspace(H, B, S, ldx))
        ws = getattr(self, "_dw1_ws", None)
        if ws is None or ws.numel() < max(n, 1) or ws.device != xb.device:
            ws = self._dw1_ws = torch.empty((max(n, 1),), dtype=torch.float32, device=xb.device)
        out = torch.empty((H, S), dtype=torch.float32, device=xb.device)
        _lib.check(lib.d2d_central_critic_dw1(H, B, S, ldx, xb.data_ptr(), dhm.data_ptr(), ws.data_ptr(), ws.numel(),
                                              out.data_ptr(), _lib.stream_ptr()), "d2d_central_critic_dw1")
        return out

    @staticmethod
    def _dw1_gemm_bm(dhm, xb):
        """_dw1_gemm with dPre's parts sample-major ([B][pH], the fused kernel's layout): [pH][S] fp32."""
        B = dhm.shape[0]
        nc = next((c for c in (64, 50, 40, 32, 25, 20, 16, 10, 8, 5, 4, 2) if B % c == 0 and B // c >= 4096), 1)
        if nc == 1:
            return torch.mm(dhm.t(), xb, out_dtype=torch.float32)
        Bc = B // nc
        a = dhm.view(nc, Bc, dhm.shape[1]).transpose(1, 2)                              # [nc][pH][Bc], strided
        return torch.bmm(a, xb.view(nc, Bc, xb.shape[1]), out_dtype=torch.float32).sum(0)

    @staticmethod
    def _dw1_gemm(dhm, xb):
        """[pH][B] x [B][S] -> fp32 [pH][S] (p split parts) with K = B (the whole sample batch): as one GEMM its output is
        a single row of tiles, so for large B the K range is split into nc chunks of a batched GEMM
        (hipBLASLt strided batches, [nc][pH][S] partials: p = 3 for the three-way dPre split) summed afterwards."""
        B = dhm.shape[1]
        nc = next((c for c in (64, 50, 40, 32, 25, 20, 16, 10, 8, 5, 4, 2) if B % c == 0 and B // c >= 4096), 1)
        if nc == 1:
            return torch.mm(dhm, xb, out_dtype=torch.float32)
        Bc = B // nc
        a = dhm.view(dhm.shape[0], nc, Bc).permute(1, 0, 2)                          # [nc][pH][Bc], strided
        return torch.bmm(a, xb.view(nc, Bc, xb.shape[1]), out_dtype=torch.float32).sum(0)

    def _chain_dev(self, A, logp_new, logp_old_tne, cycle, T, E):
        """happo_chain on the GPU (d2d_happo_chain): ratios and the sequential fp32 products in one
        kernel, logp_old read in the rollout's [T][N][E] layout."""
        from d2dhip import _lib
        lib = _lib.require_gpu()
        N = self.n_agents
        perm = torch.as_tensor(np.asarray(cycle, dtype=np.int32), device=self.device)
        M = torch.empty((N, T * E), dtype=torch.float32, device=self.device)
        A = A.contiguous()
        rc = lib.d2d_happo_chain(N, T, E, A.data_ptr(), logp_new.data_ptr(), logp_old_tne.data_ptr(), perm.data_ptr(),
                                 M.data_ptr(), _lib.stream_ptr())
        _lib.check(rc, "d2d_happo_chain")
        return M

    def _update_epoch(self, ro, upd):
        if upd is None:
            return self._epoch_fused(ro)
        x, acts, logp_old = upd
        return self._epoch(ro, x, acts, logp_old)

    def train(self, num_iter, num_episodes=4, n_epoch=4, test_freq=100):
        from d2dhip import _lib
        _lib.refuse_ablation("D2DPPO.train()")
        scores_episode = []
        score_test_list = []
        policy_loss_list = []
        value_loss_list = []
        for iter in range(num_iter):
            ro = self._rollout(num_episodes)
            scores = ro.scores
            scores_episode += scores
            upd = self._update_state(ro)
            for epoch in range(n_epoch):
                ploss_agents, value_loss = self._update_epoch(ro, upd)
                policy_loss_list.append(ploss_agents)
                value_loss_list.append(value_loss)
                if iter % test_freq == 0:
                    score_test, jains, channel_loss, avg_rewards = self.test(50)
                    score_test_list.append(score_test)
                    print(f"Iteration: {iter}, Epoch: {epoch}, score rollout: {np.mean(scores)} "
                          f"Score test: {(score_test, jains, channel_loss, avg_rewards)}")
                    if np.max(score_test_list) == score_test:
                        if self.save_path is not None:
                            self.save(self.save_path)
                    if (score_test == 1) & (self.early_stopping):
                        return scores_episode, score_test_list, policy_loss_list, value_loss_list
        return scores_episode, score_test_list, policy_loss_list, value_loss_list
