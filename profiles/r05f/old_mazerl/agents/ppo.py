"""PPO actor-critic (config 5): agents/ppo_agent.py:13-253 and lib/trainers/ppo_trainer.py:15-141.

ActorCriticNet  same layers / names as the reference (conv stem + two 1574->1024->512 MLP heads).
calculate_returns / calculate_advantages   per-episode discounted returns (Python float64 loop
                in the reference, then float32 and normalised with the unbiased std) and
                normalised advantages (:170-186).
ppo_losses      clipped surrogate (clip 0.3), entropy bonus, value MSE (:188-203). The reference
                feeds log-probs of shape [b] (new) and [b,1] (old), so the ratio broadcasts to
                [b,b] and the surrogate is the mean over all (i,j) pairs — reproduced as is
                (SURVEY-style quirk, documented in DESIGN.md).
optimize_model  ppo_steps passes over unshuffled minibatches, total = policy + 0.5 * value,
                clip_grad_norm_(0.5), AdamW with 3 groups (actor lr, critic lr, conv mean) (:206-237).
PPOAgent        single-env drop-in with the reference constructor (do_episode/optimize_model/
                evaluate); evaluate() advances the observation (the reference keeps the first
                one, SURVEY Q16 — deliberately not copied).
"""
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
import torch.optim as optim

from .linear import GraphSafeLinear

WINDOW = (15, 15)


class ActorCriticNet(nn.Module):
    def __init__(self, in_channels=3, n_observations=6, n_actions=4, h_channels=32, hidden_dim=1024):
        super().__init__()
        self.in_channels = in_channels
        self.conv = nn.Sequential(nn.Conv2d(in_channels, h_channels, kernel_size=3, stride=1, padding=1),
                                  nn.LeakyReLU(), nn.MaxPool2d(2, 2))
        d0 = h_channels * (WINDOW[0] // 2) * (WINDOW[1] // 2) + n_observations

        def head(out):
            return nn.Sequential(GraphSafeLinear(d0, hidden_dim), nn.LeakyReLU(),
                                 GraphSafeLinear(hidden_dim, hidden_dim // 2), nn.LeakyReLU(),
                                 GraphSafeLinear(hidden_dim // 2, out))
        self.actor_head = head(n_actions)
        self.critic_head = head(1)

    def forward(self, x):
        s, w = x
        if w.dtype == torch.int32 and w.dim() == 2:  # packed windows: the HIP f32 stem
            from .stem import stem_features  # (Conv -> LeakyReLU -> MaxPool, no dropout)
            y = stem_features(w, s, self.conv[0], 0.0, None, 0)
        else:
            fw = self.conv(w)
            y = torch.cat((fw.view(fw.shape[0], -1), s), dim=1)
        return self.actor_head(y), self.critic_head(y)

    def act(self, state):
        logits, value = self.forward(state)
        prob = F.softmax(logits, dim=-1)
        action = torch.multinomial(prob, num_samples=1)
        return action, torch.log(prob.gather(1, action).squeeze(1)), value

    def evaluate(self, state, action):
        logits, value = self.forward(state)
        prob = F.softmax(logits, dim=-1)
        logp = F.log_softmax(logits, dim=-1).gather(1, action).squeeze(1)
        entropy = -torch.sum(prob * torch.log(prob + 1e-8), dim=1)
        return logp, value, entropy


def make_optimizer(net, actor_lr, critic_lr, capturable=False):
    """ppo_agent.py's 3-group AdamW. capturable (the graph-captured minibatch step, on the GPU):
    the flat-buffer HIP optimizer with the clip_grad_norm_ in the same launches (FlatAdamWGroups;
    MZ_PPO_TORCH_ADAMW=1: torch's capturable fused AdamW)."""
    groups = [(net.actor_head.parameters(), actor_lr), (net.critic_head.parameters(), critic_lr),
              (net.conv.parameters(), (actor_lr + critic_lr) / 2)]
    if capturable and next(net.parameters()).is_cuda and \
            os.environ.get("MZ_PPO_TORCH_ADAMW", "0") == "0":
        from .flat import FlatAdamWGroups
        return FlatAdamWGroups(net, groups)
    kw = dict(capturable=True, fused=True) if capturable else {}
    return optim.AdamW([
        {"params": net.actor_head.parameters(), "lr": actor_lr},
        {"params": net.critic_head.parameters(), "lr": critic_lr},
        {"params": net.conv.parameters(), "lr": (actor_lr + critic_lr) / 2},
    ], **kw)


def calculate_returns(rewards, gamma):
    out, acc = [], 0
    for r in reversed(rewards):
        acc = r + acc * gamma
        out.insert(0, acc)
    ret = torch.tensor(out)
    return (ret - ret.mean()) / ret.std()


def calculate_advantages(returns, values):
    adv = returns - values
    return (adv - adv.mean()) / (adv.std() + 1e-8)


class _PairSurrogate(torch.autograd.Function):
    """The reference's clipped surrogate with its [b, b] broadcast (ppo_agent.py:188-197: new
    log-probs [b] against old ones [b, 1]): mean over (j, i) of min(r a_i, clamp(r, 1-c, 1+c) a_i)
    with r = exp(lp_new[i] - lp_old[j]), as one HIP kernel (mz_pair_surrogate) that sums over j
    per column without materialising the 4 M-element pair matrix, and returns the gradient's
    column sums with it (torch.minimum splits a tie's gradient in halves, clamp passes it inside
    [1-c, 1+c] inclusive). Besides saving ~10 passes over 16.8 MB tensors per minibatch, this
    keeps the captured PPO step free of large temporaries: replayed from a HIP graph with eager
    work in between, the torch expression's gradient came out wrong at batch 2,048 on
    PyTorch-ROCm (profiles/dbg_ppo_graph.py; tests/test_ppo_gpu.py)."""

    @staticmethod
    def forward(ctx, lp_new, lp_old, adv, clip):
        from .. import _native as N
        b = lp_new.shape[0]
        lp_new, lp_old, adv = (t.contiguous().float() for t in (lp_new, lp_old, adv))
        part = torch.empty(b, dtype=torch.float32, device=lp_new.device)
        dsum = torch.empty_like(part)
        st = torch.cuda.current_stream(lp_new.device).cuda_stream
        N.check(N.load().mz_pair_surrogate(lp_new.data_ptr(), lp_old.data_ptr(), adv.data_ptr(), b,
                                           float(clip), part.data_ptr(), dsum.data_ptr(), st))
        ctx.save_for_backward(adv, dsum)
        ctx.n = b * lp_old.shape[0]
        return part.sum() / ctx.n

    @staticmethod
    def backward(ctx, g):
        adv, dsum = ctx.saved_tensors
        return adv * dsum * (g / ctx.n), None, None, None


def ppo_losses(logp_old, logp_new, advantages, entropy, returns, value_pred, entropy_coef,
               clip=0.3):
    advantages = advantages.detach()
    if logp_new.is_cuda and logp_new.dim() == 1 and logp_old.dim() == 2 and logp_old.shape[1] == 1 \
            and advantages.dim() == 1:
        surrogate = _PairSurrogate.apply(logp_new, logp_old.detach(), advantages, clip)
    else:
        ratio = (logp_new - logp_old).exp()
        s1 = ratio * advantages
        s2 = torch.clamp(ratio, min=1 - clip, max=1 + clip) * advantages
        surrogate = torch.min(s1, s2).mean()
    policy_loss = -(surrogate + entropy * entropy_coef).mean()
    value_loss = F.mse_loss(returns.unsqueeze(1), value_pred)
    return policy_loss, value_loss


class _PPOHeadLoss(torch.autograd.Function):
    """evaluate() + ppo_losses() + total = policy + 0.5 value (ppo_agent.py:55-66, 188-203,
    222-224) from the heads' outputs in three HIP launches (mz_ppo_head_loss: softmax, the
    action's log_softmax, entropy, the [b, b] clipped surrogate, value MSE, and d total / d logits,
    d total / d value computed in the same pass) instead of ~25 small torch kernels forward and
    backward. Same arithmetic in f32 (the loss sums in float64, fixed order)."""

    @staticmethod
    def forward(ctx, logits, value, action, lp_old, adv, ret, coef, clip):
        from .. import _native as N
        b = logits.shape[0]
        dev = logits.device
        logits = logits.contiguous()
        value = value.contiguous()
        action = action.reshape(-1).contiguous()
        lp_old = lp_old.reshape(-1).contiguous().float()
        adv, ret = adv.contiguous().float(), ret.contiguous().float()
        if not torch.is_tensor(coef):
            coef = torch.full((), float(coef), dtype=torch.float32, device=dev)
        scratch = torch.empty(12 * b, dtype=torch.float32, device=dev)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        dlogits = torch.empty(b, 4, dtype=torch.float32, device=dev)
        dvalue = torch.empty(b, 1, dtype=torch.float32, device=dev)
        N.check(N.load().mz_ppo_head_loss(
            logits.data_ptr(), logits.stride(0), value.data_ptr(), value.stride(0),
            action.data_ptr(), lp_old.data_ptr(), adv.data_ptr(), ret.data_ptr(), coef.data_ptr(),
            b, float(clip), scratch.data_ptr(), loss.data_ptr(), dlogits.data_ptr(), 4,
            dvalue.data_ptr(), 1, torch.cuda.current_stream(dev).cuda_stream))
        ctx.save_for_backward(dlogits, dvalue)
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        dlogits, dvalue = ctx.saved_tensors
        return dlogits * g, dvalue * g, None, None, None, None, None, None


FUSED_LOSS = os.environ.get("MZ_PPO_FUSED_LOSS", "1") != "0"


def ppo_minibatch(net, optimizer, pos, win, act, lp_old, adv, ret, entropy_coef, allreduce=None,
                  phase=None):
    """One minibatch step of optimize_model (ppo_agent.py:217-236). phase "a" / "b" split it
    around the gradient all-reduce (backward + pack / unpack + clip + step) for graph capture.
    On the GPU the loss and its gradient w.r.t. the heads' outputs come from the fused
    _PPOHeadLoss (MZ_PPO_FUSED_LOSS=0: the torch expressions)."""
    if phase != "b":
        logits, value = net((pos, win))
        if FUSED_LOSS and logits.is_cuda and logits.shape[1] == 4 and lp_old.dim() == 2:
            total = _PPOHeadLoss.apply(logits, value, act, lp_old, adv.detach(), ret,
                                       entropy_coef, 0.3)
        else:
            prob = F.softmax(logits, dim=-1)
            lp_new = F.log_softmax(logits, dim=-1).gather(1, act).squeeze(1)
            ent = -torch.sum(prob * torch.log(prob + 1e-8), dim=1)
            pl, vl = ppo_losses(lp_old, lp_new, adv, ent, ret, value, entropy_coef)
            total = pl + 0.5 * vl
        optimizer.zero_grad()
        total.backward()
        if phase == "a":
            allreduce.pack(net)
            return total.detach()
        if allreduce is not None:
            allreduce(net)
    else:
        allreduce.unpack(net)
        total = None
    if getattr(optimizer, "fused_clip", False):
        optimizer.max_norm = 0.5  # clip_grad_norm_ inside the optimizer's launches
    else:
        torch.nn.utils.clip_grad_norm_(net.parameters(), max_norm=0.5)
    optimizer.step()
    return total.detach() if total is not None else None


def optimize_model(net, optimizer, states, actions, logp, advantages, returns, entropy_coef,
                   batch_size, ppo_steps, allreduce=None, graph=None):
    """The reference iterates DataLoader(TensorDataset(...), batch_size, shuffle=False)
    (ppo_agent.py:214-216): consecutive, unshuffled minibatches with a short last one. The
    same minibatches are taken here as slices (a DataLoader over device tensors would gather
    and collate them row by row)."""
    cols = (states[0], states[1], actions.detach(), logp.detach(), advantages, returns)
    n = cols[0].shape[0]
    last = None
    for _ in range(ppo_steps):
        for i in range(0, n, batch_size):
            mb = [c[i:i + batch_size] for c in cols]
            if graph is not None and mb[0].shape[0] == graph.batch:
                last = graph.step(mb, entropy_coef)  # full minibatch: HIP graph replay
            else:
                last = ppo_minibatch(net, optimizer, *mb, entropy_coef, allreduce=allreduce)
    return last


class PPOMinibatchGraph:
    """optimize_model's full-size minibatch step (forward of both heads from packed windows,
    the clipped-surrogate / entropy / value losses, backward, clip_grad_norm_(0.5), AdamW) captured
    into HIP graphs and replayed: ~250 small kernels per minibatch are launch-bound when issued
    eagerly. One graph per minibatch location: the minibatches are fixed slices of the update
    pool's columns, so each graph reads its slice in place (no copies into static inputs); other
    inputs (rows re-gathered after a drop) go through one graph with static input buffers. All
    graphs share one memory pool (they never run concurrently). The entropy coefficient lives on
    the device. With a gradient all-reduce each location is two graphs with the one RCCL
    all-reduce between the replays (as the DQN learner, agents/dqn.py). The optimizer must be
    capturable (make_optimizer(..., capturable=True))."""

    MAX_GRAPHS = 64

    def __init__(self, net, optimizer, batch, allreduce=None, warmup=3):
        self.net, self.opt, self.batch, self.allreduce = net, optimizer, batch, allreduce
        self.warmup, self.done_eager = warmup, 0
        self.graphs = None           # key -> (graphs tuple, loss tensor)
        self.pool = None
        self.static = None
        self.coef = None
        self._coef_val = None

    @staticmethod
    def _key(mb):
        return tuple((x.data_ptr(), tuple(x.shape), tuple(x.stride())) for x in mb)

    def _capture(self, mb):
        ar = self.allreduce
        self.opt.zero_grad(set_to_none=True)
        kw = {} if self.pool is None else {"pool": self.pool}
        if ar is None:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, **kw):
                loss = ppo_minibatch(self.net, self.opt, *mb, self.coef)
            gs = (g,)
        else:
            ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            # thread-local capture: the process group's watchdog thread polls earlier collectives'
            # events, which a global-mode capture forbids
            with torch.cuda.graph(ga, capture_error_mode="thread_local", **kw):
                loss = ppo_minibatch(self.net, self.opt, *mb, self.coef, allreduce=ar, phase="a")
            with torch.cuda.graph(gb, pool=ga.pool(), capture_error_mode="thread_local"):
                ppo_minibatch(self.net, self.opt, *mb, self.coef, allreduce=ar, phase="b")
            gs = (ga, gb)
        if self.pool is None:
            self.pool = gs[0].pool()
        return gs, loss

    def step(self, mb, entropy_coef):
        dev = mb[0].device
        if self.coef is None:
            self.coef = torch.zeros((), dtype=torch.float32, device=dev)
        if self._coef_val != float(entropy_coef):  # changes once per update, not per minibatch
            self.coef.fill_(float(entropy_coef))
            self._coef_val = float(entropy_coef)
        ar = self.allreduce
        if self.done_eager < self.warmup:  # real steps on a side stream before any capture
            s = torch.cuda.Stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                out = ppo_minibatch(self.net, self.opt, *mb, self.coef, allreduce=ar)
            torch.cuda.current_stream(dev).wait_stream(s)
            self.done_eager += 1
            return out
        if self.graphs is None:
            self.graphs = {}
        key = self._key(mb)
        ent = self.graphs.get(key)
        if ent is None:
            if len(self.graphs) < self.MAX_GRAPHS:
                ent = self.graphs[key] = self._capture(mb)
            else:  # inputs at new places: copy into the static graph's buffers
                if self.static is None:
                    self.static = [torch.empty_like(x) for x in mb]
                    self.graphs["static"] = self._capture(self.static)
                for d, x in zip(self.static, mb):
                    d.copy_(x)
                ent = self.graphs["static"]
        gs, loss = ent
        gs[0].replay()
        if ar is not None:
            ar.reduce()
            gs[1].replay()
        return loss


class PPOAgent:
    def __init__(self, actor_lr, critic_lr, gamma, batch_size, ppo_steps, env, device, channels=3,
                 hidden_dim=1024, h_channels=32):
        self.env, self.device = env, device
        self.actor_lr, self.critic_lr = actor_lr, critic_lr
        self.gamma, self.batch_size, self.ppo_steps = gamma, batch_size, ppo_steps
        obs, _ = env.reset()
        n_obs = len(np.concatenate([obs[k] for k in obs if k != "window"]))
        self.agent = ActorCriticNet(channels, n_obs, env.action_space.n, h_channels, hidden_dim).to(device)
        self.optimizer = make_optimizer(self.agent, actor_lr, critic_lr)

    def _state(self, obs):
        s = torch.tensor(np.concatenate([obs[k] for k in obs if k != "window"], axis=0),
                         dtype=torch.float32, device=self.device).unsqueeze(0)
        return s, obs["window"].to(self.device).unsqueeze(0)

    def do_episode(self):
        states, actions, logps, values, rewards = [], [], [], [], []
        obs, _ = self.env.reset()
        done, ep_reward, win = False, 0, False
        while not done:
            st = self._state(obs)
            states.append(st)
            a, lp, v = self.agent.act(st)
            actions.append(a)
            logps.append(lp)
            values.append(v)
            obs, r, truncated, terminated, _ = self.env.step(a.item())
            rewards.append(r)
            ep_reward += r
            done = terminated or truncated
            win = terminated
        pos, win_t = zip(*states)
        states = (torch.cat(pos), torch.cat(win_t))
        actions = torch.cat(actions)
        logps = torch.stack(logps).reshape(-1, 1)
        values = torch.cat(values).squeeze(-1)
        returns = calculate_returns(rewards, self.gamma).to(self.device)
        adv = calculate_advantages(returns, values)
        return ep_reward, states, actions, logps, adv, returns, win

    def calculate_returns(self, rewards):
        return calculate_returns(rewards, self.gamma)

    def calculate_advantages(self, returns, values):
        return calculate_advantages(returns, values)

    def optimize_model(self, states, actions, logp, advantages, returns, entropy_coef):
        return optimize_model(self.agent, self.optimizer, states, actions, logp, advantages,
                              returns, entropy_coef, self.batch_size, self.ppo_steps)

    @torch.no_grad()
    def evaluate(self):
        self.agent.eval()
        obs, _ = self.env.reset()
        done, ep_reward = False, 0
        terminated = truncated = False
        while not done:
            logits, _ = self.agent(self._state(obs))
            a = torch.argmax(F.softmax(logits, dim=-1), dim=-1)
            obs, r, truncated, terminated, _ = self.env.step(a.item())
            done = terminated or truncated
            ep_reward += r
        self.agent.train()
        return ep_reward, terminated, truncated
