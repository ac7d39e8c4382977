"""Config 5: PPO on variable-size toroidal mazes (9 -> 40 cells = odd toroidal grids 17..79).

  python -m mazerl.train_ppo --envs 4096 --steps 600                      # 1 GPU
  torchrun --nproc-per-node 8 -m mazerl.train_ppo --envs 4096            # 32,768 over 8 GPUs

Instance i (global id) gets grid size dims[i % len(dims)]; N = 15 (reference crash Q8) is not in
the range. Prints one JSON line with training throughput and the greedy win-rate on fresh mazes.
"""
import argparse
import json

import torch

from .distributed import GradAllReduce, allreduce_sum, broadcast_params, init_from_env
from .trainers.ppo_trainer import VectorPPOTrainer
from .trainers.vector_trainer import best_of_mazes, evaluate, make_env


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--dims", default="17-79", help="odd range lo-hi or comma list")
    ap.add_argument("--algo", default="r-prim")
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--ppo-steps", type=int, default=2)
    ap.add_argument("--pool", type=int, default=32768)
    ap.add_argument("--gamma", type=float, default=0.9)
    ap.add_argument("--eval-mazes", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--eager-update", action="store_true", help="no captured minibatch step")
    ap.add_argument("--growth", default=None,
                    help="START,MAX: ToroidalVariableMazeEnv's +4 growth per win from START up to MAX "
                         "and the max-shape stop (toroidal_variable_maze_env.py:113-131, "
                         "ppo_trainer.py:96-105) instead of fixed per-instance sizes (--dims then "
                         "only sets the evaluation sizes)")
    ap.add_argument("--curriculum", default="none", choices=["none", "global", "per-instance"],
                    help="change_algorithm (ppo_trainer.py:137-141)")
    ap.add_argument("--candidates", type=int, default=6,
                    help="training mazes: each the easiest of C by McClendon difficulty of the "
                         "bordered maze (toroidal_maze_env.py:40-54); 1 = one Philox maze each")
    ap.add_argument("--no-bank", action="store_true",
                    help="build winners' new mazes inline instead of copying them from a maze bank")
    ap.add_argument("--resume", default=None, help="checkpoint to continue from (<path>.rank<r> "
                                                    "per rank when world > 1)")
    ap.add_argument("--save", default=None, help="checkpoint written after training")
    a = ap.parse_args(argv)
    if "-" in a.dims:
        lo, hi = (int(x) for x in a.dims.split("-"))
        dims = [n for n in range(lo, hi + 1, 2)]
    else:
        dims = [int(x) for x in a.dims.split(",")]
    rank, world, local = init_from_env()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    growth = tuple(int(x) for x in a.growth.split(",")) if a.growth else None
    env = make_env(a.envs, [growth[0]] if growth else dims, toroidal=True, algorithm=a.algo,
                   seed=0x5EED0000 + rank * a.envs, device=dev, done_list=False, reward64=True,
                   window=False, window_bits=True, candidates=a.candidates,
                   max_dim=max(growth[1] if growth else 0, max(dims)))
    tr = VectorPPOTrainer(env, dev, gamma=a.gamma, batch_size=a.batch, ppo_steps=a.ppo_steps,
                          pool_size=a.pool, seed=a.seed + 7919 * rank, use_graph=not a.eager_update,
                          bank=not a.no_bank, curriculum=None if a.curriculum == "none" else a.curriculum,
                          growth=growth, algorithm=a.algo, bank_candidates=a.candidates,
                          allreduce=GradAllReduce() if world > 1 else None)
    if world > 1:
        broadcast_params(tr.net)
    ck = (lambda p: p if world == 1 else f"{p}.rank{rank}")  # noqa: E731
    if a.resume:
        from .checkpoint import load_checkpoint
        load_checkpoint(ck(a.resume), tr)
    secs = tr.train(a.steps, log_every=100 if rank == 0 else 0,
                    log=(lambda r: print(json.dumps(r), flush=True)) if rank == 0 else None)
    if a.save:
        from .checkpoint import save_checkpoint
        save_checkpoint(ck(a.save), tr)
    st = allreduce_sum(torch.tensor([tr.episodes, tr.wins], dtype=torch.float64, device=dev))
    if rank == 0:
        rate, k = evaluate(tr, a.eval_mazes, dims, a.algo, seed=0x7E570000, eps=0.0, toroidal=True,
                           device=dev)
        # new mazes as the reference's toroidal env picks them: the easiest of 6 by the McClendon
        # difficulty of the bordered maze (toroidal_maze_env.py:40-54), scored on the GPU
        mz6 = best_of_mazes(a.eval_mazes, dims, a.algo, seed=0x7E580000, device=dev, toroidal=True)
        rate6, _ = evaluate(tr, a.eval_mazes, dims, a.algo, seed=0x7E580000, eps=0.0,
                            toroidal=True, device=dev, mazes=mz6)
        print(json.dumps({"config": "ppo toroidal variable", "envs_per_gpu": a.envs, "n_gpus": world,
                          "dims": [dims[0], dims[-1]], "vector_steps": tr.stopped_at or a.steps, "train_seconds": secs,
                          "train_env_steps_per_s": a.envs * (tr.stopped_at or a.steps) * world / secs,
                          "episodes": int(st[0]), "wins": int(st[1]), "updates": tr.updates,
                          "seed": a.seed, "acting": "f32 (ActorCriticNet.act as the reference)",
                          "win_rate_greedy": rate, "win_rate_greedy_best_of_6": rate6,
                          "candidates": a.candidates, "stopped_at": tr.stopped_at,
                          "schedule": tr.schedule.summary() if tr.schedule is not None else None,
                          "eval_mazes": a.eval_mazes, "eval_steps": k}), flush=True)
    env.close()


if __name__ == "__main__":
    main()
