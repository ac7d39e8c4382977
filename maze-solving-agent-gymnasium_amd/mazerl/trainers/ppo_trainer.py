"""Vectorised PPO (config 5: variable-size toroidal mazes) — PPOTrainer.train/PPOAgent.do_episode
(lib/trainers/ppo_trainer.py:62-99, agents/ppo_agent.py:143-169) over B instances at once.

Per vector step, with no host round trip (csrc/mz_ppo.hip):
  act      the f32 ActorCriticNet forward (HIP f32 conv stem from the window bits + f32 GEMMs —
           the reference acts in f32, ppo_agent.py:55-68), then mz_ppo_act: softmax, one draw per
           instance, the draw's log-prob, and the record of (obs6, window bits, action, log-prob,
           value) at the instance's step index t[i] of [B, L] episode buffers in HBM (L = more
           than the longest possible episode, episode_bound);
  step     the env step (float64 rewards: the reference's Python floats);
  scan     mz_ppo_scan: the reward at t[i], t[i] += 1; for finished episodes the counters, t[i] = 0
           and the list of finished episodes with their pool offsets (instance order);
  finish   mz_ppo_finish: per finished episode calculate_returns / calculate_advantages
           (:171-186; returns in float64, normalised with the unbiased std) and its rows appended
           to the update pool (fixed-capacity SoA columns in HBM);
  reset    winners get new mazes (update_maze), truncated instances restart theirs; with a
           curriculum / growth schedule (schedule.py) the winners' next algorithm
           (change_algorithm, ppo_trainer.py:137-141) and size (+4 growth, the max-shape stop,
           :96-105) first.
The pool's appended-rows total is copied to the host one step late (it only grows), so the
"pool holds `pool_size` rows" test costs no synchronisation; when it passes, the update runs:
optimize_model over the first pool_size rows (ppo_steps passes of unshuffled minibatches: clipped
surrogate incl. the reference's [b, b] ratio broadcast, entropy bonus with the linear 1e-2 -> 5e-4
schedule, 0.5 * value MSE, clip_grad_norm 0.5), and the rest moves to the front of the pool.
1-step episodes (NaN returns: torch.std of one element) never reach the pool; any other row with a
non-finite advantage or return is dropped at update time (the reference would train on NaN).
"""
import time

import torch
import torch.nn.functional as F

from .. import _native as N
from ..agents.ppo import ActorCriticNet, PPOMinibatchGraph, make_optimizer, optimize_model
from .schedule import WinSchedule, curriculum_rule


def episode_bound(max_dim, toroidal):
    """Record-buffer length L: more than the longest possible episode of any maze up to max_dim.
    An episode ends at the latest on step max_steps + 1 (base_maze_env.py:205-208), max_steps =
    ceil(((N-1)^2 - 1) * len / CE) with CE = (N-1) * ((N-1) // 2) - 1 and len = the solution's
    squares (simple_maze_env.py:52-58), at most the maze's open squares: 2 c - 1 for c cells,
    c = ((N-1)/2)^2 euclidean and ((N+1)/2)^2 on the torus (generated on the (N+2)^2 bordered grid,
    so len / CE can exceed 1 there and (N-1)^2 + 2 is not a bound). +2: the float rounding of
    len / CE and the step that reports truncation."""
    best = 0
    for n in range(5, int(max_dim) + 1, 2):
        c = ((n + 1) // 2) ** 2 if toroidal else ((n - 1) // 2) ** 2
        ce = (n - 1) * ((n - 1) // 2) - 1
        a = (n - 1) ** 2 - 1
        best = max(best, -(-a * (2 * c - 1) // ce) + 2)
    return best


def pool_update(net, opt, cols, coef, batch_size, ppo_steps, allreduce=None, graph=None):
    """optimize_model on one pool's rows `cols` = (obs6, window bits or f32 window, action,
    log-prob, advantage, return). Rows with a non-finite advantage / return are dropped; with a
    gradient all-reduce every rank keeps the smallest kept count over the ranks, so all ranks run
    the same minibatch schedule (the same collective count and graph-replay / eager split).
    Returns the number of rows trained on."""
    s6, w, a, lp, adv, ret = cols
    P = s6.shape[0]
    keep = torch.isfinite(adv) & torch.isfinite(ret)
    n_keep = keep.sum().reshape(1)
    if allreduce is not None:
        import torch.distributed as dist
        dist.all_reduce(n_keep, op=dist.ReduceOp.MIN)
    n_keep = int(n_keep.item())
    if n_keep < P or not bool(keep[:n_keep].all()):
        rows = torch.nonzero(keep).flatten()[:n_keep]
        s6, w, a, lp, adv, ret = (x.index_select(0, rows) for x in (s6, w, a, lp, adv, ret))
    optimize_model(net, opt, (s6, w), a[:, None], lp[:, None], adv, ret, coef, batch_size,
                   ppo_steps, allreduce=allreduce, graph=graph)
    return n_keep


class VectorPPOTrainer:
    def __init__(self, env, device, actor_lr=3e-4, critic_lr=1e-4, gamma=0.9, batch_size=2048,
                 ppo_steps=4, pool_size=65536, hidden_dim=1024, h_channels=32, seed=0,
                 allreduce=None, use_graph=True, bank=True, pool_capacity=None, curriculum=False,
                 growth=None, algorithm="r-prim", bank_candidates=1):
        """curriculum (False | True / "global" | "per-instance"), growth ((start, max_dim): the
        variable-size envs' +4 per win and the max-shape stop), algorithm (the initial mazes'),
        bank_candidates (best-of-C replacement mazes): schedule.py, VectorOffPolicyTrainer."""
        self.env = env
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("VectorPPOTrainer runs on the GPU (libmazerl HIP kernels)")
        from ..gemm_tuning import enable as _tuned_gemms
        _tuned_gemms(self.device)  # the tuned f32 GEMM choices (gemm_tuning.py)
        if env.window_bits is None or env.reward64 is None:
            raise ValueError("VectorPPOTrainer needs an env with window_bits=True, reward64=True")
        rule = curriculum_rule(curriculum)
        self.curriculum = rule
        self.schedule = (WinSchedule(env, rule, growth, None, algorithm)
                         if (rule is not None or growth is not None) else None)
        self.stopped_at = None
        if bank:
            # winners' new mazes (update_maze) copied from a bank built ahead of time on a side
            # stream, one per grid size of the variable-size env, instead of built inline
            dims = getattr(env, "dims_in_use", None)
            if self.schedule is not None and self.schedule.growth is not None:
                dims = self.schedule.sizes()
            env.enable_bank(algorithms=[0, 1, 2] if rule else None, dims=dims,
                            candidates=bank_candidates)
        torch.manual_seed(seed)
        self.net = ActorCriticNet(3, 6, 4, h_channels, hidden_dim).to(self.device)
        # the update reads the pool's packed windows through the HIP stem and replays a captured
        # minibatch step (PPOMinibatchGraph)
        self.opt = make_optimizer(self.net, actor_lr, critic_lr, capturable=use_graph)
        self.graph = PPOMinibatchGraph(self.net, self.opt, batch_size, allreduce) if use_graph else None
        self.gamma, self.batch_size, self.ppo_steps = gamma, batch_size, ppo_steps
        self.pool_size = int(pool_size)
        self.allreduce = allreduce
        self.seed = int(seed)
        self.counter = 0
        B = env.num_envs
        self.L = L = episode_bound(env.max_dim, env.toroidal)
        kw = dict(device=self.device)
        # per-instance episode records [B, L]
        self.b_s6 = torch.zeros(B, L, 6, dtype=torch.float32, **kw)
        self.b_w = torch.zeros(B, L, 22, dtype=torch.int32, **kw)
        self.b_a = torch.zeros(B, L, dtype=torch.int64, **kw)
        self.b_lp = torch.zeros(B, L, dtype=torch.float32, **kw)
        self.b_v = torch.zeros(B, L, dtype=torch.float32, **kw)
        self.b_r = torch.zeros(B, L, dtype=torch.float64, **kw)
        self.t = torch.zeros(B, dtype=torch.int32, **kw)
        self.act_out = torch.zeros(B, dtype=torch.int32, **kw)
        # the update pool. Fill bound at an update: < pool_size + the rows the w <= 5 vector steps
        # between a check's issue and its use can append (an instance appends <= L + w rows over
        # w steps: one episode of <= L steps ending in the window plus episodes inside it);
        # 2 B L also leaves room for ranks that fill at different rates
        self.cap = int(pool_capacity or self.pool_size + 2 * B * L)
        C = self.cap
        self.p_s6 = torch.zeros(C, 6, dtype=torch.float32, **kw)
        self.p_w = torch.zeros(C, 22, dtype=torch.int32, **kw)
        self.p_a = torch.zeros(C, dtype=torch.int64, **kw)
        self.p_lp = torch.zeros(C, dtype=torch.float32, **kw)
        self.p_adv = torch.zeros(C, dtype=torch.float32, **kw)
        self.p_ret = torch.zeros(C, dtype=torch.float32, **kw)
        self.fin_id = torch.zeros(B, dtype=torch.int32, **kw)
        self.fin_off = torch.zeros(B, dtype=torch.int64, **kw)
        self.fin_len = torch.zeros(B, dtype=torch.int32, **kw)
        self.fin_count = torch.zeros(1, dtype=torch.int32, **kw)
        self.pool_fill = torch.zeros(1, dtype=torch.int64, **kw)
        self.pool_total = torch.zeros(1, dtype=torch.int64, **kw)
        # episodes, wins, dropped 1-step episodes, record-buffer overflows (an error, _update)
        self.stats = torch.zeros(4, dtype=torch.int64, **kw)
        self._total_host = torch.zeros(1, dtype=torch.int64, pin_memory=True)
        self._total_ev = None
        self.calls = 0  # _due() calls; a pool check is issued every check_every of them
        self.check_every = 1 if allreduce is None else 4
        self.consumed = 0
        self.updates = 0
        self.rows_trained = 0
        self.lib = N.load()

    @property
    def supports_bits(self):
        return True

    @property
    def episodes(self):
        return int(self.stats[0])

    @property
    def wins(self):
        return int(self.stats[1])

    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def _cols(self, lo, hi):
        return (self.p_s6[lo:hi], self.p_w[lo:hi], self.p_a[lo:hi], self.p_lp[lo:hi],
                self.p_adv[lo:hi], self.p_ret[lo:hi])

    @torch.no_grad()
    def _act(self):
        """ActorCriticNet.act in f32 for every instance + the record at t[i] (mz_ppo_act)."""
        env = self.env
        logits, value = self.net((env.obs6, env.window_bits))
        logits, value = logits.contiguous(), value.contiguous()
        B = env.num_envs
        N.check(self.lib.mz_ppo_act(
            logits.data_ptr(), logits.stride(0), value.data_ptr(), value.stride(0),
            env.obs6.data_ptr(), env.window_bits.data_ptr(), B, self.L,
            self.seed & 0xFFFFFFFFFFFFFFFF, self.counter & 0xFFFFFFFFFFFFFFFF, self.t.data_ptr(),
            self.b_s6.data_ptr(), self.b_w.data_ptr(), self.b_a.data_ptr(), self.b_lp.data_ptr(),
            self.b_v.data_ptr(), self.act_out.data_ptr(), self._stream()))
        self.counter += 1
        return logits, value

    def _scan_finish(self, reward64=None, terminated=None, truncated=None):
        """The step's outcome (default: the env's output tensors) -> records, finished episodes
        -> pool."""
        env, B, L, st = self.env, self.env.num_envs, self.L, self._stream()
        r64 = env.reward64 if reward64 is None else reward64
        term = env.terminated if terminated is None else terminated
        trunc = env.truncated if truncated is None else truncated
        N.check(self.lib.mz_ppo_scan(
            r64.data_ptr(), term.data_ptr(), trunc.data_ptr(), B, L,
            self.t.data_ptr(), self.b_r.data_ptr(), self.fin_id.data_ptr(), self.fin_off.data_ptr(),
            self.fin_len.data_ptr(), self.fin_count.data_ptr(), self.pool_fill.data_ptr(),
            self.pool_total.data_ptr(), self.stats.data_ptr(), st))
        N.check(self.lib.mz_ppo_finish(
            self.b_r.data_ptr(), self.b_s6.data_ptr(), self.b_w.data_ptr(), self.b_a.data_ptr(),
            self.b_lp.data_ptr(), self.b_v.data_ptr(), B, L, self.fin_id.data_ptr(),
            self.fin_off.data_ptr(), self.fin_len.data_ptr(), self.fin_count.data_ptr(),
            float(self.gamma), self.cap, self.p_s6.data_ptr(), self.p_w.data_ptr(),
            self.p_a.data_ptr(), self.p_lp.data_ptr(), self.p_adv.data_ptr(),
            self.p_ret.data_ptr(), st))

    def _due(self):
        """True when the pool held >= pool_size rows when the last check was issued (the host
        copy of the appended total lands while the next vector step runs; it only grows, so a
        late look never overshoots). A check is issued every `check_every` vector steps (1 on
        one rank; with a gradient all-reduce every 4th step, and the copy is the MIN over the
        ranks, so all ranks decide alike with one small collective per 4 vector steps: the pool's
        capacity covers the 2 L rows per instance that the delay can add)."""
        due = False
        if self._total_ev is not None:
            self._total_ev.synchronize()
            due = int(self._total_host[0]) - self.consumed >= self.pool_size
            self._total_ev = None
        if self.calls % self.check_every == 0:
            src = self.pool_total
            if self.allreduce is not None:
                import torch.distributed as dist
                src = self.pool_total.clone()
                dist.all_reduce(src, op=dist.ReduceOp.MIN)
            self._total_host.copy_(src, non_blocking=True)
            self._total_ev = torch.cuda.Event()
            self._total_ev.record()
        self.calls += 1
        return due

    def _update(self, frac):
        P = self.pool_size
        k = torch.div(self.pool_fill, P, rounding_mode="floor")
        # [update count, -record overflows, -pool over capacity]: one MIN all-reduce gives the
        # ranks' common update count and the MAX of both error flags, so every rank raises
        # together (a rank raising alone would leave the others blocked in pool_update's
        # collectives)
        chk = torch.cat([k, -self.stats[3:4], -(self.pool_fill > self.cap).to(torch.int64)])
        if self.allreduce is not None:
            import torch.distributed as dist
            dist.all_reduce(chk, op=dist.ReduceOp.MIN)
        # one synchronisation per update: the fill, the update count over the ranks, overflows
        fill, k, over, overcap = (int(x) for x in torch.cat([self.pool_fill, chk]).cpu())
        over, overcap = -over, -overcap
        if over:
            raise RuntimeError(f"PPO episode records overflowed: {over} episodes reached "
                               f"L = {self.L} steps (mz_ppo_scan stats[3], max over the ranks)")
        if overcap:
            raise RuntimeError(f"PPO pool overflow: more rows than the capacity {self.cap} on a "
                               f"rank (this rank: {fill}; raise pool_capacity)")
        coef = 1e-2 - (1e-2 - 5e-4) * frac  # ppo_trainer.py:73
        for j in range(k):
            self.rows_trained += pool_update(self.net, self.opt, self._cols(j * P, (j + 1) * P),
                                             coef, self.batch_size, self.ppo_steps,
                                             allreduce=self.allreduce, graph=self.graph)
            self.updates += 1
        rest = fill - k * P
        if k and rest:
            for col in self._cols(0, self.cap):
                col[:rest].copy_(col[k * P:fill].clone() if rest > k * P else col[k * P:fill])
        self.pool_fill.fill_(rest)
        self.consumed += k * P

    def vector_step(self, frac=0.0):
        env = self.env
        self._act()
        env.step(self.act_out)
        self._scan_finish()
        sch = self.schedule
        if sch is not None:  # change_algorithm for the winners (ppo_trainer.py:95)
            won = env.terminated.bool()
            sch.before_reset(won)
        env.reset_done(regen_won=True)
        if sch is not None:  # update_maze's sizes, the max-shape stop (:96-105)
            sch.after_reset(won)
        if self._due():
            self._update(frac)

    @property
    def algo(self):
        return None if self.schedule is None else self.schedule.maze_algo

    def train(self, vector_steps, log_every=0, log=print):
        t0 = time.perf_counter()
        sch = self.schedule
        for k in range(vector_steps):
            self.vector_step(frac=k / max(1, vector_steps))
            # the max-shape stop (ppo_trainer.py:104-105) once every instance reached it
            if sch is not None and sch.growth is not None and (k + 1) % 32 == 0 and sch.all_retired():
                self.stopped_at = k + 1
                break
            if log_every and (k + 1) % log_every == 0 and log:
                log(dict(step=k + 1, episodes=self.episodes, wins=self.wins, updates=self.updates,
                         seconds=round(time.perf_counter() - t0, 2)))
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    # ---- checkpoint / resume (mazerl/checkpoint.py) -------------------------------------------
    _REC = ("b_s6", "b_w", "b_a", "b_lp", "b_v", "b_r")
    _POOL = ("p_s6", "p_w", "p_a", "p_lp", "p_adv", "p_ret")

    def state_dict(self):
        """The run between two vector steps: the net, the optimizer (moments, step, per-group
        learning rates), the in-flight episodes' records (only each instance's first t[i] rows of
        the [B, L] buffers), the update pool's filled rows, the counters and the env."""
        torch.cuda.synchronize(self.device)
        t = self.t.clone()
        live = torch.arange(self.L, device=self.device)[None, :] < t[:, None].long()
        fill = int(self.pool_fill.item())
        o = self.opt
        if hasattr(o, "exp_avg"):
            ost = {k: getattr(o, k).clone() for k in ("exp_avg", "exp_avg_sq", "step_t", "lr_dev")}
        else:
            ost = {"torch": o.state_dict()}
        return {"format": "mazerl.VectorPPOTrainer/2", "L": self.L, "cap": self.cap,
                "schedule": None if self.schedule is None else self.schedule.state_dict(),
                "net": {k: v.clone() for k, v in self.net.state_dict().items()}, "opt": ost,
                "t": t, "records": {k: getattr(self, k)[live] for k in self._REC},
                "pool_fill": fill, "pool": {k: getattr(self, k)[:fill].clone() for k in self._POOL},
                "pool_total": self.pool_total.clone(), "stats": self.stats.clone(),
                # the appended total the next _due() reads (copied one vector step late)
                "total_host": int(self._total_host[0]) if self._total_ev is not None else None,
                "counters": {k: getattr(self, k) for k in ("seed", "counter", "consumed", "updates",
                                                           "rows_trained", "calls")},
                "env": self.env.state_dict()}

    def load_state_dict(self, sd):
        if sd.get("format") == "mazerl.VectorPPOTrainer/1":
            raise ValueError("a format-1 VectorPPOTrainer checkpoint (3 stats counters, a different "
                             "record length rule): not loadable by this version")
        if sd.get("format") != "mazerl.VectorPPOTrainer/2" or sd["L"] != self.L or sd["cap"] != self.cap:
            raise ValueError("not a VectorPPOTrainer state_dict of this shape")
        if (sd["schedule"] is None) != (self.schedule is None):
            raise ValueError("curriculum / growth differ from the saved trainer's")
        self.env.load_state_dict(sd["env"])
        if self.schedule is not None:
            self.schedule.load_state_dict(sd["schedule"])
        with torch.no_grad():
            self.net.load_state_dict(sd["net"])
        o, so = self.opt, sd["opt"]
        if "torch" in so:
            o.load_state_dict(so["torch"])
        else:
            for k, v in so.items():
                getattr(o, k).copy_(v)
        self.t.copy_(sd["t"])
        live = torch.arange(self.L, device=self.device)[None, :] < self.t[:, None].long()
        for k in self._REC:
            getattr(self, k)[live] = sd["records"][k].to(self.device)
        fill = int(sd["pool_fill"])
        for k in self._POOL:
            getattr(self, k)[:fill].copy_(sd["pool"][k])
        self.pool_fill.fill_(fill)
        self.pool_total.copy_(sd["pool_total"])
        self.stats.copy_(sd["stats"])
        for k, v in sd["counters"].items():
            setattr(self, k, int(v))
        self._total_ev = None
        if sd["total_host"] is not None:  # what the saved trainer's next _due() would have read
            self._total_host[0] = int(sd["total_host"])
            self._total_ev = torch.cuda.Event()
            self._total_ev.record()

    @torch.no_grad()
    def greedy(self, obs6, window, bits=None):
        """PPOAgent.evaluate's action (ppo_agent.py:239-252): argmax of softmax(logits), f32."""
        logits, _ = self.net((obs6, bits if bits is not None else window))
        return torch.argmax(F.softmax(logits, dim=-1), dim=-1)
