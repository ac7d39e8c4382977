"""What a winner's next maze is, in the vectorised trainers: the win branch of the reference's
trainers (NeuralOffPolicyTrainer.train, lib/trainers/off_policy_trainer.py:190-214; PPOTrainer.train,
lib/trainers/ppo_trainer.py:84-105), per vector step and on the device (no host round trip):

  change_algorithm(num_win)   off_policy_trainer.py:302-310 / ppo_trainer.py:137-141 — the 5th win
                              switches the maze algorithm to prim&kill, the 10th to dfs (the DQN
                              trainer also multiplies epsilon_decay by 3 / 4 there);
  env.update_maze()           the winner's new maze: same size (simple_maze_env.py:81-94), or the
                              variable-size envs' growth (simple_variable_maze_env.py:93-112,
                              toroidal_variable_maze_env.py:113-131): shape + 4 while it stays
                              <= max_shape, otherwise NO new maze (only `random.shuffle(self.mazes)`);
  the max-shape stop          off_policy_trainer.py:210-212 / ppo_trainer.py:104-105: training ends
                              once the env's shape reaches max_shape after a win.

The reference trains ONE agent on ONE env, so `num_win` counts that agent's wins and
`BaseMazeEnv.ALGORITHM` is a class attribute every env shares (base_maze_env.py:17,60-64). Two
vectorised readings of change_algorithm:

  "global" (default)   the learner is the agent: its wins over all instances are counted in
                       instance order within a vector step, the winner holding global win number
                       k gets an algorithm-k maze (r-prim before the 5th win, prim&kill from the
                       5th, dfs from the 10th — the class-wide ALGORITHM at that point of the
                       reference's sequence), and epsilon_decay (one per agent) is multiplied by 3
                       / 4 in the vector step that holds the 5th / 10th win. Instances that have
                       not won since keep the maze (and algorithm) they have.
  "per-instance"       every instance is a trainer of its own: its own win count drives its
                       algorithm and its own epsilon_decay (a per-instance tensor).

With N data-parallel ranks (rank r owns global instances [r B, (r + 1) B)) the learner's wins are
counted over every rank's instances in global instance order: each vector step the ranks exchange
their winner counts (one all-gather of N int64s), and a winner's global win number is the wins of
all earlier vector steps + the wins of the lower ranks in this step + its rank within its own
shard — the same numbers one process holding all N B instances would assign, so every rank
switches algorithms and multiplies epsilon_decay at the same vector step. The max-shape stop
likewise waits for every rank's instances (a MIN all-reduce of the retired flag every 32 vector
steps): a rank that stopped alone would leave the others' learner collectives unmatched.

Growth is per instance (the size belongs to the env, and every instance is an env): an instance's
k-th new maze on a win is start + 4 k while that is <= max_dim; a win at a size whose + 4 would pass
max_dim keeps the maze; an instance whose size reaches max_dim on a win is `retired` (the
reference's trainer returns there). The vectorised trainers stop once every instance is retired
(retired instances keep stepping their last maze until then — a batch cannot drop rows).
"""
import torch
import torch.distributed as dist

from ..vector_env import ALGOS


def _world():
    """(rank, world size) of the default process group, (0, 1) without one."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1

RULES = ("global", "per-instance")


def curriculum_rule(curriculum):
    """curriculum argument -> None | "global" | "per-instance" (True = "global")."""
    if curriculum is None or curriculum is False:
        return None
    if curriculum is True:
        return "global"
    if curriculum not in RULES:
        raise ValueError(f"curriculum rule {curriculum!r}: one of {RULES}")
    return curriculum


def growth_sizes(start, max_dim):
    """The sizes update_maze walks through from `start`: start, start + 4, ... <= max_dim."""
    return list(range(int(start), int(max_dim) + 1, 4))


class WinSchedule:
    def __init__(self, env, curriculum=None, growth=None, learner=None, algorithm="r-prim"):
        self.env, self.learner = env, learner
        self.rule = curriculum_rule(curriculum)
        self.rank, self.world = _world()
        dev, B = env.device, env.num_envs
        if isinstance(algorithm, str):
            a = torch.full((B,), ALGOS[algorithm], dtype=torch.uint8, device=dev)
        else:
            a = torch.as_tensor(algorithm, device=dev).to(torch.uint8).clone()
            if a.numel() != B:
                raise ValueError("one algorithm per instance")
        self.algo = a                        # algorithm of each instance's next maze
        self.maze_algo = a.clone()           # algorithm of each instance's current maze
        self.total_wins = torch.zeros((), dtype=torch.int64, device=dev)
        self.inst_wins = torch.zeros(B, dtype=torch.int32, device=dev)
        # new mazes handed to winners per algorithm id (index_add: no host synchronisation)
        self.new_mazes = torch.zeros(3, dtype=torch.int64, device=dev)
        self.growth = None
        if growth is not None:
            start, mx = (int(x) for x in growth)
            if start % 2 == 0 or mx % 2 == 0 or start > mx or mx > env.max_dim:
                raise ValueError(f"growth {growth}: odd start <= odd max_dim <= the env's max_dim")
            self.growth = (start, mx)
            self.dim = torch.full((B,), start, dtype=torch.int32, device=dev)
            self.next_dim = torch.empty(B, dtype=torch.uint8, device=dev)
            self.retired = torch.zeros(B, dtype=torch.bool, device=dev)
            self._set_next()
            env.set_regen_dims(self.next_dim)

    def sizes(self):
        """Maze sizes a bank must hold for this schedule (None: the env's own)."""
        return growth_sizes(*self.growth) if self.growth else None

    def _set_next(self):
        mx = self.growth[1]
        self.next_dim.copy_(torch.where(self.dim + 4 <= mx, self.dim + 4, 0).to(torch.uint8))

    def before_reset(self, term):
        """change_algorithm for this vector step's winners (`term`: the step's terminated flags,
        device) — sets the algorithm of their next maze before the reset regenerates it."""
        t = term.bool()
        w = t.to(torch.int32)
        if self.rule is None:  # growth only: the win counts (summary) still advance
            if self.growth is not None:
                self.total_wins += w.sum()
                self.inst_wins += w
            return
        dfs, pk = ALGOS["dfs"], ALGOS["prim&kill"]
        if self.rule == "global":
            # global win numbers of this step's winners, in global instance order: the wins of
            # the lower ranks' shards first (data-parallel), then this shard's in instance order
            mine = w.sum().to(torch.int64)
            if self.world > 1:
                parts = [torch.zeros(1, dtype=torch.int64, device=mine.device)
                         for _ in range(self.world)]
                dist.all_gather(parts, mine.view(1))
                cnt = torch.cat(parts)
                off, step_wins = cnt[:self.rank].sum(), cnt.sum()
            else:
                off, step_wins = 0, mine
            rank = self.total_wins + off + torch.cumsum(w, 0)
            na = torch.where(rank >= 10, dfs, torch.where(rank >= 5, pk, self.algo.long()))
            self.algo = torch.where(t, na.to(torch.uint8), self.algo)
            before = self.total_wins.clone()
            self.total_wins += step_wins
            self.inst_wins += w
            L = self.learner
            if L is not None and hasattr(L, "eps_decay"):
                if not torch.is_tensor(L.eps_decay):
                    L.eps_decay = torch.tensor(float(L.eps_decay), device=self.env.device)
                after = self.total_wins
                f = torch.where((before < 5) & (after >= 5), 3.0, 1.0) * \
                    torch.where((before < 10) & (after >= 10), 4.0, 1.0)
                L.eps_decay.mul_(f)
        else:
            self.inst_wins += w
            self.total_wins += w.sum()
            iw = self.inst_wins
            L = self.learner
            if L is not None and hasattr(L, "eps_decay"):
                if not torch.is_tensor(L.eps_decay) or L.eps_decay.dim() == 0:
                    L.eps_decay = torch.full((self.env.num_envs,), float(L.eps_decay),
                                             device=self.env.device)
                L.eps_decay.mul_(torch.where(t & (iw == 5), 3.0, torch.where(t & (iw == 10), 4.0, 1.0)))
            na = torch.where(iw >= 10, dfs, torch.where(iw >= 5, pk, self.algo.long()))
            self.algo = torch.where(t, na.to(torch.uint8), self.algo)
        self.env.set_algorithm(self.algo)

    def after_reset(self, term):
        """The winners' new sizes / algorithms after the reset built their mazes; the next sizes
        and the retirements (the max-shape stop)."""
        t = term.bool()
        if self.growth is None:
            if self.rule is not None:
                self.maze_algo = torch.where(t, self.algo, self.maze_algo)
                self.new_mazes.index_add_(0, self.algo.long(), t.to(torch.int64))
            return
        moved = t & (self.next_dim > 0)  # winners that got a maze of the next size
        self.new_mazes.index_add_(0, self.algo.long(), moved.to(torch.int64))
        self.dim = torch.where(moved, self.next_dim.to(torch.int32), self.dim)
        self.maze_algo = torch.where(moved, self.algo, self.maze_algo)
        self.retired |= t & (self.dim >= self.growth[1])
        self._set_next()

    def all_retired(self):
        """The max-shape stop: every instance of every rank retired (one MIN all-reduce with N
        ranks — every rank calls this at the same vector steps)."""
        if self.growth is None:
            return False
        done = self.retired.all().to(torch.int32).view(1)
        if self.world > 1:
            dist.all_reduce(done, op=dist.ReduceOp.MIN)
        return bool(done.item())

    def summary(self):
        """Host-side counts (one synchronisation)."""
        names = ["r-prim", "dfs", "prim&kill"]  # ids: vector_env.ALGOS
        out = {"rule": self.rule, "total_wins": int(self.total_wins),  # (global: all ranks')
               "instances_per_algorithm": dict(zip(
                   names, torch.bincount(self.maze_algo.long(), minlength=3).tolist())),
               "new_mazes_per_algorithm": dict(zip(names, self.new_mazes.tolist())),
               "wins_per_instance_median": float(self.inst_wins.float().median())}
        if self.growth is not None:
            sizes = growth_sizes(*self.growth)
            cnt = torch.bincount((self.dim - self.growth[0]) // 4, minlength=len(sizes)).tolist()
            out.update(growth=list(self.growth), instances_per_size=dict(zip(sizes, cnt)),
                       retired=int(self.retired.sum()))
        return out

    _STATE = ("algo", "maze_algo", "total_wins", "inst_wins", "new_mazes")

    def state_dict(self):
        sd = {k: getattr(self, k).clone() for k in self._STATE}
        sd["rule"] = self.rule
        if self.growth is not None:
            sd.update(growth=list(self.growth), dim=self.dim.clone(), retired=self.retired.clone())
        return sd

    def load_state_dict(self, sd):
        if sd["rule"] != self.rule or (sd.get("growth") is None) != (self.growth is None):
            raise ValueError("curriculum rule / growth differ from the saved schedule's")
        for k in self._STATE:
            setattr(self, k, sd[k].to(self.env.device).clone())
        if self.growth is not None:
            self.dim = sd["dim"].to(self.env.device).clone()
            self.retired = sd["retired"].to(self.env.device).clone()
            self._set_next()
            self.env.set_regen_dims(self.next_dim)
        self.env.set_algorithm(self.algo)
