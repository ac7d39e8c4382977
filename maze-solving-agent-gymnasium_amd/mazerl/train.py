"""Vectorised DQN/DDQN training + win-rate evaluation (configs 2-4 of BASELINE.json).

  python -m mazerl.train --envs 65536 --dim 81 --variant ddqn --steps 400          # 1 GPU
  torchrun --nproc-per-node 8 -m mazerl.train --envs 8192 --dim 81 --algo mixed    # 8 GPUs

Prints one JSON line: training throughput (env steps/s and updates/s over all ranks) and the
win-rate on fresh mazes (greedy and epsilon = eps_final, reference protocol Q14).
"""
import argparse
import json
import time

import torch

from .agents.dqn import VectorDQNLearner
from .distributed import GradAllReduce, allreduce_sum, broadcast_params, init_from_env
from .trainers.vector_trainer import VectorOffPolicyTrainer, best_of_mazes, evaluate, make_env


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536, help="instances per GPU")
    ap.add_argument("--dim", type=int, default=81)
    ap.add_argument("--algo", default="r-prim", help="r-prim | dfs | prim&kill | mixed")
    ap.add_argument("--variant", default="ddqn")
    ap.add_argument("--steps", type=int, default=400, help="vector steps")
    ap.add_argument("--updates-per-step", type=int, default=1)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--gamma", type=float, default=0.7)
    ap.add_argument("--eps-start", type=float, default=0.95)
    ap.add_argument("--eps-final", type=float, default=0.1)
    ap.add_argument("--eps-decay", type=float, default=None, help="default ((N-1)^2//2)*5 / 40")
    ap.add_argument("--capacity", type=int, default=2_000_000)
    ap.add_argument("--target-every", type=int, default=13)
    ap.add_argument("--eval-mazes", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--curriculum", default="none", choices=["none", "global", "per-instance"],
                    help="change_algorithm (off_policy_trainer.py:302-310): prim&kill from the 5th "
                         "win, dfs from the 10th, epsilon_decay *3 / *4 — counted over the learner's "
                         "wins (global, the reference's one agent) or per instance "
                         "(mazerl/trainers/schedule.py)")
    ap.add_argument("--growth", default=None,
                    help="START,MAX: the variable-size env's +4 growth per win from START up to MAX "
                         "and the max-shape stop (simple_variable_maze_env.py:93-112, "
                         "off_policy_trainer.py:210-212); --dim is then MAX")
    ap.add_argument("--candidates", type=int, default=6,
                    help="training mazes: each the easiest of C by McClendon difficulty "
                         "(base_maze_env.py:78-97); 1 = one Philox maze each")
    ap.add_argument("--log-every", type=int, default=50)
    ap.add_argument("--acting", default="x3", choices=["x3", "bf16"],
                    help="acting forward: x3 = f32-accurate bf16x3 MFMA (QAct); bf16 = bf16 head")
    ap.add_argument("--overlap", type=int, default=1,
                    help="1: updates on a side HIP stream (acting one update behind); 0: sequential")
    ap.add_argument("--resume", default=None,
                    help="checkpoint to continue from (mazerl/checkpoint.py; rank r reads "
                         "<path>.rank<r> when world > 1)")
    ap.add_argument("--save", default=None, help="checkpoint written after training (same naming)")
    return ap.parse_args(argv)


def _ck_path(path, rank, world):
    return path if world == 1 else f"{path}.rank{rank}"


def main(argv=None):
    a = parse(argv)
    rank, world, local = init_from_env()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    B = a.envs
    if a.algo == "mixed":  # config 4: algo_id = global instance id mod 3
        algo = (torch.arange(B) + rank * B) % 3
    else:
        algo = a.algo
    growth = tuple(int(x) for x in a.growth.split(",")) if a.growth else None
    if growth:
        a.dim = growth[1]
    env = make_env(B, growth[0] if growth else a.dim, algorithm=algo, seed=0x5EED0000 + rank * B,
                   device=dev, max_dim=a.dim, candidates=a.candidates, done_list=False, pos=True,
                   window=False, window_bits=True)  # acting reads the bits (agents/fused.py)
    env.set_algorithm(algo if isinstance(algo, str) else algo.to(torch.uint8))
    decay = a.eps_decay or ((a.dim - 1) * (a.dim - 1) // 2) * 5 / 40.0
    learner = VectorDQNLearner(B, dev, variant=a.variant, lr=a.lr, eps_start=a.eps_start,
                               eps_final=a.eps_final, eps_decay=decay, gamma=a.gamma,
                               batch_size=a.batch, capacity=a.capacity,
                               updates_per_step=a.updates_per_step, target_every=a.target_every,
                               allreduce=GradAllReduce() if world > 1 else None, seed=a.seed,
                               overlap=bool(a.overlap), acting=a.acting)
    if world > 1:
        broadcast_params(learner.source)
        learner.target.load_state_dict(learner.source.state_dict())
    trainer = VectorOffPolicyTrainer(env, learner, seed=a.seed + 7919 * rank,
                                     curriculum=None if a.curriculum == "none" else a.curriculum,
                                     growth=growth, algorithm=algo, bank_candidates=a.candidates)
    if a.resume:  # every rank its own shard's env / replay; the nets are identical on all ranks
        from .checkpoint import load_checkpoint
        load_checkpoint(_ck_path(a.resume, rank, world), trainer)
    secs = trainer.train(a.steps, log_every=a.log_every if rank == 0 else 0,
                         log=(lambda r: print(json.dumps(r), flush=True)) if rank == 0 else None)
    stats = torch.stack([trainer.wins, trainer.episodes]).to(torch.float64)
    allreduce_sum(stats)
    t = torch.tensor([secs], dtype=torch.float64, device=dev)
    if world > 1:
        import torch.distributed as dist
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    secs = float(t.item())
    if a.save:
        from .checkpoint import save_checkpoint
        save_checkpoint(_ck_path(a.save, rank, world), trainer)
    res = {}
    if rank == 0:
        eval_algo = "r-prim" if a.algo == "mixed" else a.algo
        greedy, kg = evaluate(learner, a.eval_mazes, a.dim, eval_algo, seed=0x7E570000, eps=0.0, device=dev)
        epsr, ke = evaluate(learner, a.eval_mazes, a.dim, eval_algo, seed=0x7E570000, eps=a.eps_final, device=dev)
        # fresh mazes as the reference's env picks them: the easiest of 6 (base_maze_env.py:78-97)
        mz6 = best_of_mazes(a.eval_mazes, a.dim, eval_algo, seed=0x7E580000, device=dev)
        g6, _ = evaluate(learner, a.eval_mazes, a.dim, eval_algo, seed=0x7E580000, eps=0.0,
                         device=dev, mazes=mz6)
        e6, _ = evaluate(learner, a.eval_mazes, a.dim, eval_algo, seed=0x7E580000,
                         eps=a.eps_final, device=dev, mazes=mz6)
        res = {
            "variant": a.variant, "envs_per_gpu": B, "n_gpus": world, "dim": a.dim, "algo": a.algo,
            "vector_steps": trainer.stopped_at or a.steps, "train_seconds": secs,
            # (the max-shape stop can end training before a.steps)
            "train_env_steps_per_s": B * (trainer.stopped_at or a.steps) * world / secs,
            "updates": learner.n_updates, "updates_per_s": learner.n_updates / secs,
            "batch": a.batch, "train_wins": int(stats[0]), "train_episodes": int(stats[1]),
            "win_rate_greedy": greedy, "win_rate_eps": epsr, "eval_eps": a.eps_final,
            "win_rate_greedy_best_of_6": g6, "win_rate_eps_best_of_6": e6,
            "eval_mazes": a.eval_mazes, "eval_steps": [kg, ke],
            "candidates": a.candidates, "stopped_at": trainer.stopped_at,
            "schedule": trainer.schedule.summary() if trainer.schedule is not None else None,
        }
        print(json.dumps(res), flush=True)
    env.close()
    return res


if __name__ == "__main__":
    main()
