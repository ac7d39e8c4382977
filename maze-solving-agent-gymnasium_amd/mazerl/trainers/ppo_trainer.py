"""Vectorised PPO (config 5: variable-size toroidal mazes) — PPOTrainer.train/PPOAgent.do_episode
(lib/trainers/ppo_trainer.py:62-99, agents/ppo_agent.py:143-169) over B instances at once.

Per vector step every instance acts (softmax sample of the actor head, log-prob, critic value —
ActorCriticNet.act) and steps; its transition goes to its own episode buffer in HBM
(obs6 f32[B,L,6], packed windows i32[B,L,22], action, log-prob, value, float64 reward; L = the
largest possible episode, (N-1)^2 + 1). When an instance's episode ends, the episode is finished
exactly like do_episode: discounted returns accumulated backwards in float64 on the GPU
(mz_discounted_returns), normalised per episode with the unbiased std, advantages = returns -
values normalised per episode; the episode's rows are appended to the update pool. When the pool
holds `pool_size` transitions, optimize_model runs ppo_steps passes over unshuffled minibatches
(clipped surrogate incl. the reference's [b,b] ratio broadcast, entropy bonus with the linear
1e-2 -> 5e-4 schedule, 0.5 * value MSE, clip_grad_norm 0.5). Winners get new mazes (update_maze),
truncated instances restart theirs.
"""
import time

import torch
import torch.nn.functional as F

from .. import _native as N
from ..agents.ppo import ActorCriticNet, PPOMinibatchGraph, make_optimizer, optimize_model


class VectorPPOTrainer:
    def __init__(self, env, device, actor_lr=3e-4, critic_lr=1e-4, gamma=0.9, batch_size=2048,
                 ppo_steps=4, pool_size=65536, hidden_dim=1024, h_channels=32, seed=0,
                 allreduce=None, act_bf16=True, use_graph=True, bit_stem=True, bank=True):
        self.env = env
        if bank and env.device.type == "cuda":
            # winners' new mazes (update_maze) copied from a bank built ahead of time on a side
            # stream, one per grid size of the variable-size env, instead of built inline
            env.enable_bank(dims=getattr(env, "dims_in_use", None))
        self.device = torch.device(device)
        torch.manual_seed(seed)
        self.net = ActorCriticNet(3, 6, 4, h_channels, hidden_dim).to(self.device)
        # on the GPU the update reads the pool's packed windows through the HIP stem and replays
        # a captured minibatch step (PPOMinibatchGraph)
        self.on_gpu = self.device.type == "cuda"
        self.bit_stem = self.on_gpu and bit_stem
        self.opt = make_optimizer(self.net, actor_lr, critic_lr, capturable=self.on_gpu and use_graph)
        self.graph = (PPOMinibatchGraph(self.net, self.opt, batch_size, allreduce)
                      if self.on_gpu and use_graph else None)
        self.gamma, self.batch_size, self.ppo_steps = gamma, batch_size, ppo_steps
        self.pool_size = pool_size
        self.allreduce = allreduce
        self.act_bf16 = act_bf16
        B = env.num_envs
        self.L = (env.max_dim - 1) ** 2 + 2
        kw = dict(device=self.device)
        self.b_s6 = torch.zeros(B, self.L, 6, dtype=torch.float32, **kw)
        self.b_w = torch.zeros(B, self.L, 22, dtype=torch.int32, **kw)
        self.b_a = torch.zeros(B, self.L, dtype=torch.int64, **kw)
        self.b_lp = torch.zeros(B, self.L, dtype=torch.float32, **kw)
        self.b_v = torch.zeros(B, self.L, dtype=torch.float32, **kw)
        self.b_r = torch.zeros(B, self.L, dtype=torch.float64, **kw)
        self.t = torch.zeros(B, dtype=torch.int64, **kw)
        self.ar = torch.arange(B, **kw)
        self.pool = []
        self.pool_n = 0
        self.episodes = 0
        self.wins = 0
        self.updates = 0
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)
        self.fused = None
        if self.device.type == "cuda" and act_bf16:
            from ..agents.fused import FusedActorCritic
            self.fused = FusedActorCritic(self.net, seed=seed)

    @property
    def supports_bits(self):
        return self.fused is not None

    @torch.no_grad()
    def _act(self):
        env = self.env
        state = (env.obs6, env.window)
        if self.fused is not None and env.window_bits is not None:
            logits, value = self.fused(env.obs6, env.window_bits)
        elif self.act_bf16 and self.device.type == "cuda":
            with torch.autocast("cuda", dtype=torch.bfloat16):
                logits, value = self.net(state)
        else:
            logits, value = self.net(state)
        prob = F.softmax(logits.float(), dim=-1)
        a = torch.multinomial(prob, 1, generator=self.gen)
        lp = torch.log(prob.gather(1, a).squeeze(1))
        return a.squeeze(1), lp, value.float().squeeze(1)

    def _finish(self, rows):
        """do_episode's tail for the finished instances `rows` (device int64)."""
        n = int(rows.numel())
        if n == 0:
            return
        lens = self.t.index_select(0, rows)
        T = int(lens.max())
        ret = torch.zeros(n, self.L, dtype=torch.float32, device=self.device)
        rows32, lens32 = rows.to(torch.int32), lens.to(torch.int32)
        N.check(N.load().mz_discounted_returns(
            self.b_r.data_ptr(), self.L, rows32.data_ptr(), lens32.data_ptr(), n, float(self.gamma),
            ret.data_ptr(), self.L, torch.cuda.current_stream(self.device).cuda_stream))
        ret = ret[:, :T]
        mask = torch.arange(T, device=self.device)[None, :] < lens[:, None]
        cnt = lens.to(torch.float32)[:, None]

        def norm(x, eps):  # (x - mean) / (std + eps), unbiased std per episode (torch.std)
            m = (x * mask).sum(1, keepdim=True) / cnt
            var = (((x - m) * mask) ** 2).sum(1, keepdim=True) / (cnt - 1)
            return (x - m) / (var.sqrt() + eps)
        ret = norm(ret, 0.0)
        val = self.b_v.index_select(0, rows)[:, :T]
        adv = norm(ret - val, 1e-8)
        sel = mask.flatten()
        ri = rows[:, None].expand(n, T).flatten()[sel]
        ti = torch.arange(T, device=self.device)[None, :].expand(n, T).flatten()[sel]
        chunk = (self.b_s6[ri, ti], self.b_w[ri, ti], self.b_a[ri, ti], self.b_lp[ri, ti],
                 adv.flatten()[sel], ret.flatten()[sel])
        self.pool.append(chunk)
        self.pool_n += int(sel.sum())

    def _ready(self):
        """All ranks update together, each on exactly pool_size rows (equal collective counts)."""
        n = torch.tensor([self.pool_n], dtype=torch.int64, device=self.device)
        if self.allreduce is not None:
            import torch.distributed as dist
            dist.all_reduce(n, op=dist.ReduceOp.MIN)
        return int(n.item()) >= self.pool_size

    def _update(self, frac):
        cat = [torch.cat(x) for x in zip(*self.pool)]
        P = self.pool_size
        rest = [x[P:] for x in cat]
        self.pool = [tuple(rest)] if rest[0].shape[0] else []
        self.pool_n = int(rest[0].shape[0])
        s6, w, a, lp, adv, ret = (x[:P] for x in cat)
        win = w if self.bit_stem else self.env.expand_window(w)  # packed bits -> HIP stem
        coef = 1e-2 - (1e-2 - 5e-4) * frac  # ppo_trainer.py:73
        keep = (adv == adv) & (ret == ret)  # a 1-step episode has an undefined std (NaN): drop
        rows = torch.nonzero(keep).flatten()
        n_keep = torch.tensor([rows.numel()], dtype=torch.int64, device=self.device)
        if self.allreduce is not None:
            # every rank must run the same minibatch schedule (same collective count and the
            # same graph-replay / eager split): all keep the smallest kept count
            import torch.distributed as dist
            dist.all_reduce(n_keep, op=dist.ReduceOp.MIN)
        n_keep = int(n_keep.item())
        if n_keep < P:
            rows = rows[:n_keep]
            s6, win, a, lp, adv, ret = (x.index_select(0, rows) for x in (s6, win, a, lp, adv, ret))
        optimize_model(self.net, self.opt, (s6, win), a[:, None], lp[:, None], adv, ret, coef,
                       self.batch_size, self.ppo_steps, allreduce=self.allreduce, graph=self.graph)
        if self.fused is not None:
            self.fused.invalidate()  # graph replays leave the params' _version as is
        self.updates += 1

    def vector_step(self, frac=0.0):
        env = self.env
        a, lp, v = self._act()
        t = self.t
        self.b_s6[self.ar, t] = env.obs6
        self.b_w[self.ar, t] = env.window_bits
        self.b_a[self.ar, t] = a
        self.b_lp[self.ar, t] = lp
        self.b_v[self.ar, t] = v
        env.step(a.to(torch.int32))
        self.b_r[self.ar, t] = env.reward64
        self.t += 1
        term = env.terminated.bool()
        done = term | env.truncated.bool()
        rows = torch.nonzero(done).flatten()
        self._finish(rows)
        self.t.masked_fill_(done, 0)
        self.episodes += int(rows.numel())
        self.wins += int(term.sum())
        env.reset_done(regen_won=True)
        if self._ready():
            self._update(frac)

    def train(self, vector_steps, log_every=0, log=print):
        t0 = time.perf_counter()
        for k in range(vector_steps):
            self.vector_step(frac=k / max(1, vector_steps))
            if log_every and (k + 1) % log_every == 0 and log:
                log(dict(step=k + 1, episodes=self.episodes, wins=self.wins, updates=self.updates,
                         seconds=round(time.perf_counter() - t0, 2)))
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    @torch.no_grad()
    def greedy(self, obs6, window, bits=None):
        if bits is not None and self.fused is not None:
            logits, _ = self.fused(obs6, bits)
        else:
            logits, _ = self.net((obs6, window))
        return torch.argmax(F.softmax(logits.float(), dim=-1), dim=-1)
