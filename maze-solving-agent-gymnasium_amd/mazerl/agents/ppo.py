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
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
import torch.optim as optim

WINDOW = (15, 15)


class ActorCriticNet(nn.Module):
    def __init__(self, in_channels=3, n_observations=6, n_actions=4, h_channels=32, hidden_dim=1024):
        super().__init__()
        self.in_channels = in_channels
        self.conv = nn.Sequential(nn.Conv2d(in_channels, h_channels, kernel_size=3, stride=1, padding=1),
                                  nn.LeakyReLU(), nn.MaxPool2d(2, 2))
        d0 = h_channels * (WINDOW[0] // 2) * (WINDOW[1] // 2) + n_observations

        def head(out):
            return nn.Sequential(nn.Linear(d0, hidden_dim), nn.LeakyReLU(),
                                 nn.Linear(hidden_dim, hidden_dim // 2), nn.LeakyReLU(),
                                 nn.Linear(hidden_dim // 2, out))
        self.actor_head = head(n_actions)
        self.critic_head = head(1)

    def forward(self, x):
        s, w = x
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


def make_optimizer(net, actor_lr, critic_lr):
    return optim.AdamW([
        {"params": net.actor_head.parameters(), "lr": actor_lr},
        {"params": net.critic_head.parameters(), "lr": critic_lr},
        {"params": net.conv.parameters(), "lr": (actor_lr + critic_lr) / 2},
    ])


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


def ppo_losses(logp_old, logp_new, advantages, entropy, returns, value_pred, entropy_coef,
               clip=0.3):
    advantages = advantages.detach()
    ratio = (logp_new - logp_old).exp()
    s1 = ratio * advantages
    s2 = torch.clamp(ratio, min=1 - clip, max=1 + clip) * advantages
    surrogate = torch.min(s1, s2).mean()
    policy_loss = -(surrogate + entropy * entropy_coef).mean()
    value_loss = F.mse_loss(returns.unsqueeze(1), value_pred)
    return policy_loss, value_loss


def optimize_model(net, optimizer, states, actions, logp, advantages, returns, entropy_coef,
                   batch_size, ppo_steps, allreduce=None):
    """The reference iterates DataLoader(TensorDataset(...), batch_size, shuffle=False)
    (ppo_agent.py:214-216): consecutive, unshuffled minibatches with a short last one. The
    same minibatches are taken here as slices (a DataLoader over device tensors would gather
    and collate them row by row)."""
    cols = (states[0], states[1], actions.detach(), logp.detach(), advantages, returns)
    n = cols[0].shape[0]
    last = None
    for _ in range(ppo_steps):
        for i in range(0, n, batch_size):
            pos, win, act, lp_old, adv, ret = (c[i:i + batch_size] for c in cols)
            lp_new, value, ent = net.evaluate((pos, win), act)
            pl, vl = ppo_losses(lp_old, lp_new, adv, ent, ret, value, entropy_coef)
            total = pl + 0.5 * vl
            optimizer.zero_grad()
            total.backward()
            if allreduce is not None:
                allreduce(net)
            torch.nn.utils.clip_grad_norm_(net.parameters(), max_norm=0.5)
            optimizer.step()
            last = total.detach()
    return last


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
