"""iPPO — drop-in for /root/reference/algorithms/ippo.py (independent PPO:
one actor + one critic per agent on its own observation).

Same module-level API (init_weights, RNN, Policy, Value, compute_gae,
discount_rewards, PPO, iPPO), same constructor/method signatures and return
structures; the work runs agent-batched on the MI355X:
  * rollout: env kernel + agent-stacked actor/critic forward per slot
    (BatchedLearnerBase._collect), for every env of the batch at once;
  * advantages/returns: the HIP GAE scan + normalisation kernels;
  * update: one agent-stacked forward/backward and one Adam step per epoch
    for all N actors, same for the N critics — identical per-agent losses
    (ippo.py:194-217), which are independent across agents, so summing them
    leaves every agent's gradient unchanged.
"""
import os

import numpy as np
import torch
import torch.nn.functional as F

from ._core import Policy, RNN, StackedNets, Value, init_weights, make_dist  # noqa: F401
from ._learner import BatchedLearnerBase


def _gae_cpu_api(rewards, dones, values, gamma, lbda, which):
    """Module-level compute_gae / discount_rewards: reference inputs (numpy (T,N) or (T,)),
    computed by the HIP kernels, returned as CPU float32 tensors like the reference."""
    from d2dhip.gae import gae_returns
    r = np.asarray(rewards, dtype=np.float64)
    one_d = r.ndim == 1
    r2 = r.reshape(r.shape[0], -1)
    v = np.zeros_like(r2) if values is None else np.asarray(values, dtype=np.float64).reshape(r2.shape[0], -1)
    dev = torch.device("cuda")
    rt = torch.from_numpy(r2.astype(np.float32)).to(dev)[:, None, :]
    vt = torch.from_numpy(v.astype(np.float32)).to(dev)[:, None, :]
    if rt.shape[2] != vt.shape[2]:
        rt = rt[:, :, :1]
    dt = torch.from_numpy(np.asarray(dones, dtype=np.uint8)).to(dev)
    adv, ret = gae_returns(rt, vt, dt, gamma, lbda, normalize_adv=True, normalize_ret=(which == "ret_norm"))
    out = adv if which == "adv" else ret
    out = out[:, 0, :].cpu()
    return out[:, 0] if one_d else out


def compute_gae(rewards, dones, values, gamma, lbda=0.95):
    """ippo.py:92-102 (lambda-returns + one-off last element, ddof-0 normalisation)."""
    return _gae_cpu_api(rewards, dones, values, gamma, lbda, "adv")


def discount_rewards(rewards, gamma, dones, normalize=True):
    """ippo.py:104-116 (float64 recursion, float32 cast, ddof-1 normalisation)."""
    return _gae_cpu_api(rewards, dones, None, gamma, 0.0, "ret_norm" if normalize else "ret")


class PPO:
    """Per-agent object (ippo.py:120-217).  Its networks are views into the learner's
    agent-stacked parameters; select_action/evaluate/train_step keep the reference's
    single-agent semantics for direct callers."""

    def __init__(self, num_inputs, n_actions, hidden_size=128, gamma=0.99, policy_lr=1e-3, value_lr=1e-3,
                 useRNN=False, combinatorial=False, device='cpu', history_len=5, early_stopping=True):
        self.history_len = history_len
        self.useRNN = useRNN
        self.combinatorial = combinatorial
        self.early_stopping = early_stopping
        self.device = torch.device(device)
        self.n_actions = n_actions
        if not self.useRNN:
            self.policy_network = Policy(num_inputs, n_actions, hidden_size)
            self.value_network = Value(num_inputs, hidden_size)
        else:
            self.policy_network = RNN(num_inputs, n_actions, hidden_size, combinatorial=combinatorial)
            self.value_network = RNN(num_inputs, 1, hidden_size, combinatorial=False, use_activation=False)
        self.gamma = gamma
        self.policy_lr, self.value_lr = policy_lr, value_lr
        self.policy_optimizer = None
        self.value_optimizer = None

    def _opts(self):
        if self.policy_optimizer is None:
            self.policy_optimizer = torch.optim.Adam(self.policy_network.parameters(), lr=self.policy_lr)
            self.value_optimizer = torch.optim.Adam(self.value_network.parameters(), lr=self.value_lr)

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

    def train_step(self, states, actions, log_probs_old, returns, advantages, cliprange=0.1, beta=0.01):
        self._opts()
        log_probs, entropy = self.evaluate(states, actions)
        entropy = entropy.mean()
        ratio = torch.exp(log_probs - log_probs_old.to(self.device))
        adv = advantages.to(self.device)
        policy_loss = -torch.min(ratio * adv, torch.clamp(ratio, 1.0 - cliprange, 1.0 + cliprange) * adv).mean() \
            - beta * entropy
        self.policy_optimizer.zero_grad()
        policy_loss.backward()
        self.policy_optimizer.step()
        value = self.value_network(states.to(self.device)).squeeze()
        value_loss = F.mse_loss(value, returns.to(self.device), reduction='mean')
        self.value_optimizer.zero_grad()
        value_loss.backward()
        self.value_optimizer.step()
        return policy_loss.item(), value_loss.item()


class iPPO(BatchedLearnerBase):
    def __init__(self,
                 env,
                 hidden_size=128,
                 gamma=0.99,
                 policy_lr=1e-3,
                 value_lr=1e-3,
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
        self.policy_lr = policy_lr
        self.value_lr = value_lr
        self.early_stopping = early_stopping
        self.useRNN = useRNN
        self.combinatorial = combinatorial
        self.save_path = save_path
        self.device = self._resolve_device(device)
        if self.device.type != "cuda":
            import d2dhip
            d2dhip.require_gpu()
        self.agents = [PPO(num_inputs=self.env.observation_space[k].shape[0],
                           n_actions=self.env.action_space[k].n,
                           hidden_size=hidden_size,
                           gamma=gamma,
                           policy_lr=policy_lr,
                           value_lr=value_lr,
                           useRNN=useRNN,
                           combinatorial=combinatorial,
                           history_len=history_len,
                           device=self.device,
                           early_stopping=early_stopping) for k in range(self.n_agents)]
        in_dims = [env.observation_space[k].shape[0] for k in range(self.n_agents)]
        kind = "rnn" if useRNN else "mlp"
        self.policy = StackedNets([a.policy_network for a in self.agents], in_dims, kind, self.device,
                                  act=self._policy_act())
        self.value = StackedNets([a.value_network for a in self.agents], in_dims, kind, self.device, act=None)
        self.policy_optimizer = torch.optim.Adam(self.policy.parameters(), lr=policy_lr)
        self.value_optimizer = torch.optim.Adam(self.value.parameters(), lr=value_lr)
        self._setup_data_parallel(self.policy.parameters() + self.value.parameters())

    # ------------------------------------------------------------ rollouts
    # training rollouts of the fused MLP path take their values (ippo.py:308) from the first update epoch's
    # critic pass instead of a critic forward in every rollout slot: the critic's weights are the same at both
    # points, and that pass computes V(obs) of every sample anyway (d2d_ppo_critic_grad_values).  The rollout
    # slot then runs the actor-only policy kernel; GAE follows the critic pass.  D2D_DEFER_VALUES=0: per-slot values
    defer_values = os.environ.get("D2D_DEFER_VALUES", "1") != "0"

    def _defer_values_ok(self):
        return self.defer_values and not self.useRNN and self._fused_ok() and self._fused_update_ok()

    def _rollout(self, num_episodes, teacher=None, defer_values=False):
        """defer_values (train()): values and advantages are filled in by the first _epoch_fused on this rollout;
        the reference-API paths (create_rollouts, tests) keep the per-slot values."""
        defer = defer_values and teacher is None and self._defer_values_ok()
        ro = self._collect(num_episodes, train=True, want_values=not defer, teacher=teacher)
        self._phase("rollout")
        if defer:
            s = self.env.batch().spec
            ro.values = torch.empty((ro.T, s.N, ro.E), dtype=torch.float32, device=self.device)
            # the returns (discount_rewards, ippo.py:338) read no value: they are the critic pass's targets.  Every
            # agent gets the same reward (the envs broadcast |S| / the ACK), so the N normalised return columns are
            # identical: one column, viewed over the agents with stride 0
            zero = torch.zeros((ro.T, 1, ro.E), dtype=torch.float32, device=self.device)
            _, ret1 = self._gae(ro.rewards, zero, ro.dones, normalize_adv=False, layout="tce")
            ro.ret_tne = ret1.expand(ro.T, s.N, ro.E)
            ro.adv_tne = None
            ro.values_pending = True
        else:
            # values [T][N][E] as the policy kernel wrote them; adv / ret in the same layout (ippo.py:337-338)
            ro.adv_tne, ro.ret_tne = self._gae(ro.rewards, ro.values, ro.dones, layout="tce")
        self._phase("gae")
        return ro

    def create_rollouts(self, num_episodes=4):
        """Reference return structure (ippo.py:343): obs list [N] of (T, in_i), actions np (T, N[, C]),
        log_probs (T, N), returns (T, N), values np (T, N), advantages (T, N), scores, dones.
        With n_envs > 1 the sample axis is the env-major concatenation of all episodes."""
        ro = self._rollout(num_episodes)
        return self._reference_view(ro)

    def _reference_view(self, ro):
        s = self.env.batch().spec
        N = s.N
        obs = ro.obs_f32.permute(2, 1, 0, 3).reshape(N, ro.E * ro.T, -1)
        obs_list = [obs[k, :, : s.obs_len[k]] for k in range(N)]
        acts = ro.actions.permute(1, 0, 2).reshape(ro.E * ro.T, N)
        if self.kind == "comb":
            from ._core import unpack_actions
            acts = unpack_actions(acts, s.C)
        actions = acts.cpu().numpy()
        log_probs = self._seq(ro.logp).t().cpu()
        values = self._seq(ro.values).t().cpu().numpy().astype(np.float64)
        dones = [bool(d) for d in ro.dones.cpu().tolist()] * ro.E
        return (obs_list, actions, log_probs, ro.ret.t().cpu(), values, ro.adv.t().cpu(), ro.scores, dones)

    # -------------------------------------------------------------- update
    def _epoch(self, x, acts, logp_old, adv, ret, cliprange=0.1, beta=0.01):
        """One reference epoch (ippo.py:418-426) for all agents at once."""
        log_probs, entropy = self._evaluate(x, acts)
        ratio = torch.exp(log_probs - logp_old)
        surr1 = ratio * adv
        surr2 = torch.clamp(ratio, 1.0 - cliprange, 1.0 + cliprange) * adv
        policy_loss = -torch.min(surr1, surr2).mean(1) - beta * entropy.mean(1)          # [N]
        self.policy_optimizer.zero_grad()
        policy_loss.sum().backward()
        self._reduce_grads(self.policy.parameters())
        self.policy_optimizer.step()
        value = self.value.forward(x)[..., 0]
        value_loss = ((value - ret) ** 2).mean(1)                                          # [N]
        self.value_optimizer.zero_grad()
        value_loss.sum().backward()
        self._reduce_grads(self.value.parameters())
        self.value_optimizer.step()
        return policy_loss.detach(), value_loss.detach()

    def _epoch_fused(self, ro, cliprange=0.1, beta=0.01):
        """The same epoch on the fused HIP update kernels: gradients of every agent's policy loss
        and value loss straight from the rollout buffers, written into .grad; Adam in torch."""
        from d2dhip.update import actor_grads, critic_grads
        pp, vp = self.policy.params, self.value.params
        kind = "comb" if self.combinatorial else "chsel"
        B = ro.T * ro.E
        sv = None
        critic_first = bool(getattr(ro, "values_pending", False))
        if critic_first:
            # first epoch on a deferred-values rollout: the critic pass first, writing V(obs) of every sample --
            # the rollout critic's values (same weights) -- then its Adam step, then GAE for the actor (the two
            # optimizers are independent, so the order of the two updates does not change either)
            _, sv = critic_grads({k: v.data for k, v in vp.items()}, ro.obs, ro.ret_tne.permute(0, 2, 1),
                                 grads=self._grad_buffers(vp), values=ro.values.permute(0, 2, 1))
            self._phase("critic_grad")
            self._reduce_grads(self.value.parameters())
            self._phase("allreduce")
            self.value_optimizer.step()
            self._phase("adam")
            ro.adv_tne, _ = self._gae(ro.rewards, ro.values, ro.dones, normalize_ret=False, layout="tce")
            ro.values_pending = False
            self._phase("gae")
        if self.useRNN:  # GRU policies / critics: BPTT over the padded training windows (gru_kernels.hip)
            from d2dhip import gru
            _, sa = gru.grads({k: v.data for k, v in pp.items()}, ro.obs, self._gru_kind(), self.history_len, ro.L,
                              ro.adv_tne.permute(0, 2, 1), actions=ro.actions, logp_old=ro.logp.permute(0, 2, 1),
                              clip=cliprange, beta=beta, grads=self._grad_buffers(pp))
        else:
            _, sa = actor_grads({k: v.data for k, v in pp.items()}, ro.obs, ro.actions, ro.logp.permute(0, 2, 1),
                                ro.adv_tne.permute(0, 2, 1), kind, clip=cliprange, beta=beta,
                                grads=self._grad_buffers(pp))
        self._phase("actor_grad")
        self._reduce_grads(self.policy.parameters())
        self._phase("allreduce")
        self.policy_optimizer.step()
        self._phase("adam")
        if critic_first:  # (the critic ran first on this epoch)
            pass
        elif self.useRNN:
            from d2dhip import gru
            _, sv = gru.grads({k: v.data for k, v in vp.items()}, ro.obs, None, self.history_len, ro.L,
                              ro.ret_tne.permute(0, 2, 1), grads=self._grad_buffers(vp))
        else:
            _, sv = critic_grads({k: v.data for k, v in vp.items()}, ro.obs, ro.ret_tne.permute(0, 2, 1),
                                 grads=self._grad_buffers(vp))
        if not critic_first:
            self._phase("critic_grad")
            self._reduce_grads(self.value.parameters())
            self._phase("allreduce")
            self.value_optimizer.step()
            self._phase("adam")
        return -(sa[:, 0] + beta * sa[:, 1]) / B, sv[:, 0] / B

    def _update_epoch(self, ro, upd):
        if upd is None:
            return self._epoch_fused(ro)
        x, acts, logp_old = upd
        return self._epoch(x, acts, logp_old, ro.adv, ro.ret)

    def train(self, num_iter, n_epoch=4, num_episodes=4, test_freq=100):
        from d2dhip import _lib
        _lib.refuse_ablation("iPPO.train()")
        scores_episode = []
        score_test_list = []
        policy_loss_list = []
        value_loss_list = []
        for iter in range(num_iter):
            ro = self._rollout(num_episodes, defer_values=True)
            scores = ro.scores
            scores_episode += scores
            upd = self._update_state(ro)
            for epoch in range(n_epoch):
                pl, vl = self._update_epoch(ro, upd)
                # the reference appends the losses of the last agent of its loop (ippo.py:425-426)
                policy_loss_list.append(pl[-1].item())
                value_loss_list.append(vl[-1].item())
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
