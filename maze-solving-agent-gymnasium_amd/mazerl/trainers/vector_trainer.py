"""Vectorised off-policy trainer and win-rate evaluation on VectorMazeEnv.

VectorOffPolicyTrainer.train() is NeuralOffPolicyTrainer.train (lib/trainers/off_policy_trainer.py
:144-225) over B instances at once. Per vector step:
  greedy  = argmax Q_source(obs)   fused HIP conv stem on the window bits + bf16 MFMA GEMMs
                                                      (agents/fused.py, dqn_agent.py:113-116),
             over the instances whose epsilon draw of this step says "greedy" only
  step    = fused epsilon-greedy act + env step       (one k_step launch, per-instance epsilon)
  replay  <- (s, a, r, s') for every instance, s' = the step's (terminal) observation; terminal
             transitions bootstrap like the reference's
  bookkeeping: steps_done += 1, = 0 on a win (off_policy_trainer.py:192); wins/episodes counters
  auto-reset: winners get a new maze (update_maze, :202), truncated instances restart the same
             maze (reset, :153) — one flag-scan kernel; new mazes are copied from a bank of
             pre-generated mazes (refilled in bulk on a side stream; bank_candidates=6: each the
             easiest of 6 by McClendon difficulty, the reference env's generate_maze selection,
             base_maze_env.py:78-97); change_algorithm / growth / the max-shape stop: schedule.py
  K learner updates (replay ratio), target sync / cosine step per update count.
evaluate() is NeuralOffPolicyTrainer.test(new=True)/infer (:228-299): fresh mazes, one episode
each, win = terminated; greedy (eps = 0) or the reference's epsilon protocol (Q14).
"""
import os
import time

import torch

from ..vector_env import ALGOS, VectorMazeEnv
from .schedule import WinSchedule, curriculum_rule


class VectorOffPolicyTrainer:
    """curriculum: False | True / "global" | "per-instance" (change_algorithm, schedule.py);
    growth: None | (start, max_dim) — the variable-size envs' +4 growth per win and the max-shape
    stop (schedule.py; make the env with make_env(B, start, max_dim=max_dim)); algorithm: the
    initial mazes' algorithm (str or per-instance ids), the curriculum's base;
    bank_candidates: best-of-C maze bank (1 = one Philox maze per slot)."""

    def __init__(self, env, learner, seed=0, regen_won=True, curriculum=False, allreduce_stats=None,
                 bank=True, fused=True, growth=None, algorithm="r-prim", bank_candidates=1,
                 track_wins=False):
        self.env, self.learner = env, learner
        # inst_wins (per-instance win counts) is kept by the win schedule; track_wins keeps it
        # without one (one more launch per vector step)
        self.track_wins = bool(track_wins)
        rule = curriculum_rule(curriculum)
        self.schedule = (WinSchedule(env, rule, growth, learner, algorithm)
                         if (rule is not None or growth is not None) else None)
        if regen_won and bank:
            # winners' new mazes come from a bank refilled on a side stream (VectorMazeEnv.
            # enable_bank): a maze build is a ~1 ms serial chain that would stall the step
            dims = getattr(env, "dims_in_use", None)
            if self.schedule is not None and self.schedule.growth is not None:
                dims = self.schedule.sizes()
            env.enable_bank(algorithms=[0, 1, 2] if rule else None, dims=dims,
                            candidates=bank_candidates)
        self.seed = seed
        # fused: the per-step bookkeeping and the replay push as HIP launches (mz_trainer_tick,
        # mz_replay_push) instead of ~25 torch ops; False keeps the torch path (A/B, tests)
        self.fused = bool(fused)
        self.regen_won = regen_won
        self.curriculum = rule
        self.allreduce_stats = allreduce_stats
        dev = env.device
        self.wins = torch.zeros((), dtype=torch.int64, device=dev)
        self.episodes = torch.zeros((), dtype=torch.int64, device=dev)
        self.inst_wins = torch.zeros(env.num_envs, dtype=torch.int32, device=dev)
        self.counter = 0
        self.stopped_at = None  # vector step of the max-shape stop (growth), if it came
        self._eps = None  # the next step's epsilon, computed at the end of the previous step
        self.history = []

    @property
    def algo(self):
        """Algorithm id of each instance's current maze (None without a schedule)."""
        return None if self.schedule is None else self.schedule.maze_algo

    def _expand(self, bits):
        return self.env.expand_window(bits)

    def vector_step(self):
        env, L = self.env, self.learner
        # epsilon of this step's fused act (fixed by the previous step's bookkeeping)
        eps = self._eps if self._eps is not None else L.epsilon()
        self._eps = None
        # (eps, seed, counter) of this step's fused act: the acting forward runs over the rows
        # that will act greedily only (the row list was issued at the end of the previous step)
        greedy = L.greedy(env.obs6, env.window, env.window_bits, act=(eps, self.seed, self.counter))
        rp = L.replay
        ring = self.fused and hasattr(rp, "push_state") and env.window_bits is not None and \
            env.device.type == "cuda"
        if ring:  # the replay rows' state half, straight from the observation the step replaces
            rp.push_state(env.obs6, env.window_bits)
        else:
            s6, sw = env.obs6.clone(), env.window_bits.clone()
        env.step_act(eps=eps, greedy=greedy, seed=self.seed, counter=self.counter)
        self.counter += 1
        # (a curriculum changes epsilon_decay on the device: the torch bookkeeping path)
        tick = getattr(L, "tick", None) if self.fused and not self.curriculum else None
        # steps_done (+1, 0 on a win), wins / episodes, the next step's epsilon and its greedy-row
        # list — issued now, so that its count reaches the host while the stream runs the push
        # and the resets queued behind it
        self._eps = tick(env.terminated, env.truncated, self.wins, self.episodes, self.seed,
                         self.counter) if tick is not None else None
        if self._eps is None:
            term = env.terminated.bool()
            L.steps_done += 1
            L.steps_done.masked_fill_(term, 0)
            if hasattr(L, "prepare_greedy"):
                self._eps = L.epsilon()
                L.prepare_greedy(self._eps, self.seed, self.counter)
            self.wins += term.sum()
            self.episodes += (term | env.truncated.bool()).sum()
        sch = self.schedule
        if sch is not None:  # change_algorithm for this step's winners (off_policy_trainer.py:201)
            won = env.terminated.bool()
            self.inst_wins += won.to(torch.int32)
            sch.before_reset(won)
        elif self.track_wins:
            self.inst_wins += env.terminated.to(torch.int32)
        if ring:
            rp.push_rest(env.actions, env.reward, env.obs6, env.window_bits)
        else:
            rp.push(s6, sw, env.actions, env.reward, env.obs6, env.window_bits)
        env.reset_done(regen_won=self.regen_won)
        if sch is not None:  # update_maze's sizes, the max-shape stop (:202-212)
            sch.after_reset(won)
        # with an overlapped learner the updates run on its side stream; the next push (one row
        # per instance) is kept out of their sample range
        return L.update(self._expand, reserve=env.num_envs)

    def train(self, vector_steps, log_every=0, log=print):
        t0 = time.perf_counter()
        prio = os.environ.get("MZ_ACT_PRIORITY")
        if prio is None or self.env.device.type != "cuda":
            return self._train(vector_steps, log_every, log, t0)
        # acting / env work on a stream of its own priority (the learner's side stream keeps the
        # default one): the small per-step kernels get CUs ahead of the update's
        outer = torch.cuda.current_stream(self.env.device)
        if getattr(self, "_act_stream", None) is None:
            self._act_stream = torch.cuda.Stream(self.env.device, priority=int(prio))
        s = self._act_stream
        s.wait_stream(outer)
        with torch.cuda.stream(s):
            secs = self._train(vector_steps, log_every, log, t0)
        outer.wait_stream(s)
        return secs

    def state_dict(self):
        """Checkpoint of the whole run (mazerl/checkpoint.py): this trainer's counters, the env
        (VectorMazeEnv.state_dict) and the learner (VectorDQNLearner.state_dict). train() calls
        after a load_state_dict continue exactly as further train() calls on the saved trainer
        would have."""
        L = self.learner
        return {"format": "mazerl.VectorOffPolicyTrainer/2", "seed": self.seed,
                "counter": self.counter, "wins": self.wins.clone(), "episodes": self.episodes.clone(),
                "inst_wins": self.inst_wins.clone(), "curriculum": self.curriculum,
                "regen_won": self.regen_won, "history": list(self.history),
                "schedule": None if self.schedule is None else self.schedule.state_dict(),
                "learner": L.state_dict(), "env": self.env.state_dict()}

    def load_state_dict(self, sd):
        fmt = sd.get("format")
        if fmt == "mazerl.VectorOffPolicyTrainer/1":
            raise ValueError("a format-1 VectorOffPolicyTrainer checkpoint (before the win "
                             "schedule, round 5): not loadable by this version")
        if fmt != "mazerl.VectorOffPolicyTrainer/2":
            raise ValueError("not a VectorOffPolicyTrainer state_dict")
        if sd["curriculum"] != self.curriculum or bool(sd["regen_won"]) != bool(self.regen_won) \
                or (sd["schedule"] is None) != (self.schedule is None):
            raise ValueError("curriculum / growth / regen_won differ from the saved trainer's")
        self.env.load_state_dict(sd["env"])
        self.learner.load_state_dict(sd["learner"])
        if self.schedule is not None:
            self.schedule.load_state_dict(sd["schedule"])
        self.seed, self.counter = int(sd["seed"]), int(sd["counter"])
        self.wins.copy_(sd["wins"])
        self.episodes.copy_(sd["episodes"])
        self.inst_wins.copy_(sd["inst_wins"])
        self.history = list(sd["history"])
        self._eps = None

    def _train(self, vector_steps, log_every, log, t0):
        # the next step's epsilon and its issued greedy-row list are recomputed on entry: the
        # caller may have changed steps_done (a reload, a reset) since the last train() call
        self._eps = None
        rows = getattr(self.learner, "_rows", None)
        if rows is not None:
            rows._issued = None
        sch = self.schedule
        for k in range(vector_steps):
            loss = self.vector_step()
            # the max-shape stop (off_policy_trainer.py:210-212) once every instance reached it
            if sch is not None and sch.growth is not None and (k + 1) % 32 == 0 and sch.all_retired():
                self.stopped_at = k + 1
                break
            if log_every and (k + 1) % log_every == 0:
                torch.cuda.synchronize()
                rec = dict(step=k + 1, wins=int(self.wins), episodes=int(self.episodes),
                           loss=float(loss) if loss is not None else None,
                           eps_mean=float(self.learner.epsilon().mean()),
                           seconds=round(time.perf_counter() - t0, 2))
                self.history.append(rec)
                if log:
                    log(rec)
        if hasattr(self.learner, "finish"):
            self.learner.finish()
        torch.cuda.synchronize()
        return time.perf_counter() - t0


def make_env(num_envs, dims, toroidal=False, algorithm="r-prim", seed=0x5EED0000, device=None,
             max_dim=None, candidates=1, **kw):
    """VectorMazeEnv whose instance i gets maze size dims[i % len(dims)] (variable-size configs);
    max_dim: the handle's pitch (default max(dims); a growth schedule needs its max size);
    candidates > 1: every initial maze the easiest of `candidates` (the reference env's
    generate_maze selection, base_maze_env.py:78-97 — its constructors draw the first maze so)."""
    dims = [dims] if isinstance(dims, int) else list(dims)
    env = VectorMazeEnv(num_envs, dims[0], toroidal=toroidal, enrich=True, device=device,
                        max_dim=max(max(dims), int(max_dim or 0)), algorithm=algorithm, seed=seed,
                        generate=len(dims) == 1, candidates=candidates, **kw)
    env.dims_in_use = sorted(set(dims))  # (a maze bank for the winners then holds every size)
    if len(dims) > 1:
        ids = torch.arange(num_envs, device=env.device)
        for j, n in enumerate(dims):
            sel = ids[ids % len(dims) == j]
            if sel.numel():
                algo = algorithm if isinstance(algorithm, str) else torch.as_tensor(algorithm)[sel.cpu()]
                env.generate(env_ids=sel.to(torch.int32), algorithm=algo, dim=n, seed=seed,
                             candidates=candidates)
        env.set_algorithm(algorithm if isinstance(algorithm, str) else torch.as_tensor(algorithm).to(torch.uint8))
        env.reset()
    return env


def maze_algorithms(num_mazes, seed, algos=("r-prim", "prim&kill", "dfs")):
    """NeuralOffPolicyTrainer.test(new=True)'s per-maze `random.choice(OffPolicyTrainer.ALGOS)`
    (off_policy_trainer.py:231-233), drawn from a Python random.Random(seed): a list of names."""
    import random
    rng = random.Random(seed)
    return [rng.choice(list(algos)) for _ in range(num_mazes)]


def best_of_mazes(num_mazes, dim, algorithm="r-prim", seed=0x7E57, device=None, candidates=6,
                  toroidal=False):
    """The reference's maze selection for new mazes (BaseMazeEnv.generate_maze,
    base_maze_env.py:78-97; toroidal: ToroidalMazeEnv.generate_maze, toroidal_maze_env.py:40-54,
    scored on the bordered maze): per maze, `candidates` generated mazes of the same size and
    algorithm, keep the one with the smallest McClendon difficulty (strict <: the first minimum).
    `algorithm` is one name or a per-maze list of names (test(new=True)'s random choice); `dim` is
    one size or a list (maze k gets dim[k % len], as make_env / evaluate assign them). The
    candidates are GPU-generated (Philox) and scored on the GPU in one launch (mz_difficulty_batch,
    one workgroup per maze; host mz_difficulty for the mazes it declines).
    Returns (grids uint8 [n, D, D], start_goal [n, 4], sizes int [n]) with D = the largest size
    (a smaller maze in the top-left corner) for evaluate(mazes=...) / load_mazes per size."""
    import numpy as np
    from ..difficulty import difficulty_batch
    dims = [dim] if isinstance(dim, int) else list(dim)
    n, C = int(num_mazes), int(candidates)
    size_of = [dims[k % len(dims)] for k in range(n)]
    algo_of = [algorithm] * n if isinstance(algorithm, str) else list(algorithm)
    if len(algo_of) != n:
        raise ValueError("one algorithm per maze")
    cand = VectorMazeEnv(n * C, size_of[0], toroidal=toroidal, enrich=True, device=device,
                         max_dim=max(dims), algorithm=algo_of[0], seed=seed, done_list=False,
                         pos=False, window=False, window_bits=False,
                         generate=len(set(size_of)) == 1 and len(set(algo_of)) == 1)
    if len(set(size_of)) > 1 or len(set(algo_of)) > 1:
        groups = {}
        for k in range(n):
            groups.setdefault((size_of[k], algo_of[k]), []).extend(range(k * C, k * C + C))
        for (sz, al), ids in sorted(groups.items()):
            cand.generate(env_ids=torch.tensor(ids, dtype=torch.int32, device=cand.device),
                          algorithm=al, dim=sz, seed=seed)
    d = difficulty_batch(cand).reshape(n, C)
    pick = d.argmin(axis=1)  # first minimum (NaN-free: a log domain error raises on the host)
    D = max(dims)
    grids = np.zeros((n, D, D), np.uint8)
    sg = np.zeros((n, 4), np.int32)
    for k in range(n):
        i = k * C + int(pick[k])
        q = cand.query(i)
        g = cand.grid(i)
        grids[k, :g.shape[0], :g.shape[1]] = g
        sg[k] = (q["start_r"], q["start_c"], q["goal_r"], q["goal_c"])
    cand.close()
    return grids, sg, np.asarray(size_of, np.int32)


def load_selected(env, mazes):
    """Load best_of_mazes' (grids, start_goal[, sizes]) into env instances 0..n-1, one
    mz_load_mazes call per size."""
    import numpy as np
    grids, sg = mazes[0], mazes[1]
    sizes = mazes[2] if len(mazes) > 2 else np.full(len(grids), grids.shape[1], np.int32)
    for sz in sorted(set(int(x) for x in sizes)):
        ids = np.nonzero(sizes == sz)[0].astype(np.int32)
        env.load_mazes(np.ascontiguousarray(grids[ids, :sz, :sz]), sg[ids], env_ids=ids)
    env.reset()


def snapshot_mazes(env, ids):
    """The listed instances' current mazes as best_of_mazes returns them (grids uint8 [n, D, D],
    start_goal int32 [n, 4], sizes [n]; D = the largest): the mazes the reference's env keeps in
    `env.mazes` — the first one and each win's update_maze replacement (simple_maze_env.py:81-94)
    — are, for a trained instance, the mazes it holds over training; evaluate(mazes=...) replays
    them as test(n, new=False) does (update_visited_maze(remove=True), :96-116)."""
    import numpy as np
    ids = [int(i) for i in ids]
    qs = [env.query(i) for i in ids]
    D = max(q["n"] for q in qs)
    grids = np.zeros((len(ids), D, D), np.uint8)
    sg = np.zeros((len(ids), 4), np.int32)
    sizes = np.zeros(len(ids), np.int32)
    for k, (i, q) in enumerate(zip(ids, qs)):
        g = env.grid(i)
        grids[k, :g.shape[0], :g.shape[1]] = g
        sg[k] = (q["start_r"], q["start_c"], q["goal_r"], q["goal_c"])
        sizes[k] = q["n"]
    return grids, sg, sizes


def steps_done_epsilon(learner, num_mazes, instances=None):
    """The reference's test-time epsilon (test() acts through DQNAgent.get_action, dqn_agent.py:
    104-119: eps = eps_final + (eps_start - eps_final) * exp(-steps_done / decay), steps_done += 1
    per action, never reset during test): a callable k -> per-maze epsilon after k actions, each
    evaluation maze k continuing the steps_done (and epsilon decay) of training instance
    k mod B. Instances run their test episodes side by side here; the reference plays them one
    after another on one counter."""
    sd0 = learner.steps_done.detach().float()
    B = sd0.numel()
    idx = (torch.arange(num_mazes, device=sd0.device) % B if instances is None else
           torch.as_tensor(instances, dtype=torch.long, device=sd0.device))  # (seen mazes: their own)
    sd0 = sd0[idx]
    dec = learner.eps_decay
    dec = dec[idx] if torch.is_tensor(dec) and dec.dim() > 0 else torch.full_like(sd0, float(dec))
    e0, e1 = float(learner.eps_start), float(learner.eps_final)

    def eps(k):
        return e1 + (e0 - e1) * torch.exp(-(sd0 + float(k)) / dec)
    eps.start_mean = float((e1 + (e0 - e1) * torch.exp(-sd0 / dec)).mean())
    return eps


@torch.no_grad()
def evaluate(learner, num_mazes, dim, algorithm="r-prim", seed=0x7E57, eps=0.0, toroidal=False,
             device=None, max_vector_steps=None, mazes=None, return_won=False):
    """Fraction of `num_mazes` fresh mazes solved in one episode (terminated before truncation).
    `dim` may be a list of sizes (instance i gets dim[i % len]). `mazes` = best_of_mazes' output
    to play instead of generated ones (the reference's best-of-6 selection). `eps` is a number or
    a callable k -> per-maze epsilon tensor for the k-th action (steps_done_epsilon).
    Returns (rate, vector steps) or, with return_won, (rate, vector steps, won bool [n] on the
    host)."""
    bits = getattr(learner, "supports_bits", False)
    if not isinstance(algorithm, str) and mazes is None:
        raise ValueError("a per-maze algorithm list needs the mazes: pass best_of_mazes(...)'s "
                         "output as mazes= (evaluate generates one algorithm's mazes itself)")
    algo0 = algorithm if isinstance(algorithm, str) else "r-prim"
    env = make_env(num_mazes, dim, toroidal=toroidal, algorithm=algo0, seed=seed,
                   device=device, done_list=False, pos=False, window=not bits, window_bits=True)
    if mazes is not None:
        load_selected(env, mazes)
    dim = max(dim) if not isinstance(dim, int) else dim
    finished = torch.zeros(num_mazes, dtype=torch.bool, device=env.device)
    won = torch.zeros(num_mazes, dtype=torch.bool, device=env.device)
    limit = max_vector_steps or (dim - 1) * (dim - 1) + 2  # > any max_steps
    k = 0
    while k < limit:
        greedy = learner.greedy(env.obs6, env.window, env.window_bits)
        acts = env.act(eps=eps(k) if callable(eps) else eps, greedy=greedy, seed=seed, counter=k)
        acts = torch.where(finished, torch.full_like(acts, -1), acts)
        env.step(acts)
        term = env.terminated.bool()
        won |= term & ~finished
        finished |= term | env.truncated.bool()
        k += 1
        if k % 32 == 0 and bool(finished.all()):
            break
    rate = float(won.float().mean())
    env.close()
    if return_won:
        return rate, k, won.cpu().numpy()
    return rate, k
