"""Maze-generation metric suite (reference generation_algos_metrics_evaluations.py, README table
"1000 mazes 40x40"): per algorithm, N generated mazes on the 81x81 grid, then

  MD / Max D   mean / max McClendon difficulty   (ComplexityEvaluation.difficulty_of_maze)
  MC           mean McClendon complexity          (complexity_of_maze)
  ML, MDE, MDs mean L, DE, D of the solution path (MetricsCalculator.calculate_L/_DE/_D)

Generation and L/DE/D run on the GPU (mz_generate_ex, mz_maze_metrics); the McClendon values
run in libmazerl's host C++ (mz_maze_complexity, networkx-order restatement) on a thread pool.
With rng="cpython" the mazes are exactly the reference's for random.seed(seed + i).

  python -m mazerl.metrics --mazes 1000 --dim 81 [--rng cpython] [--seed 0]
"""
import argparse
import ctypes as C
import json
import os
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import _native as N
from .vector_env import ALGOS, VectorMazeEnv


def _mcclendon(args):
    g, s, goal = args
    d, c = C.c_double(), C.c_double()
    rc = N.load().mz_maze_complexity(g.ctypes.data, g.shape[0], g.shape[1], int(s[0]), int(s[1]),
                                     int(goal[0]), int(goal[1]), C.byref(d), C.byref(c))
    return (d.value, c.value) if rc == 0 else (float("nan"), float("nan"))


def generation_metrics(algorithm, mazes=1000, dim=81, rng="cpython", seed=0, device=None,
                       threads=None):
    env = VectorMazeEnv(mazes, dim, enrich=False, generate=False, device=device)
    env.generate(algorithm=algorithm, seed=seed, rng=rng)
    m = env.maze_metrics().cpu().numpy()
    meta = env.meta().cpu().numpy()
    jobs = [(env.grid(i), (meta[i, 1], meta[i, 2]), (meta[i, 3], meta[i, 4])) for i in range(mazes)]
    env.close()
    with ThreadPoolExecutor(threads or min(16, os.cpu_count() or 1)) as ex:
        dc = np.array(list(ex.map(_mcclendon, jobs)))
    return {"MD": float(np.nanmean(dc[:, 0])), "Max D": float(np.nanmax(dc[:, 0])),
            "MC": float(np.nanmean(dc[:, 1])), "ML": float(m[:, 0].mean()),
            "MDE": float(m[:, 1].mean()), "MDs": float(m[:, 2].mean()), "mazes": mazes,
            "grid": dim, "rng": rng}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--mazes", type=int, default=1000)
    ap.add_argument("--dim", type=int, default=81)
    ap.add_argument("--rng", default="cpython", choices=["cpython", "philox"])
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    for algo in ("dfs", "r-prim", "prim&kill"):
        t0 = time.perf_counter()
        r = generation_metrics(algo, a.mazes, a.dim, a.rng, a.seed + 10**7 * ALGOS[algo])
        r["algorithm"] = algo
        r["seconds"] = round(time.perf_counter() - t0, 2)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
