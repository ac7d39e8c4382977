#!/usr/bin/env python3
"""Golden fixture metrics.npz: the reference's maze-metric suite on the golden euclidean mazes
(tests/golden/gen_euclid.npz) — what generation_algos_metrics_evaluations.py computes per maze:

  ComplexityEvaluation(maze, start, goal).difficulty_of_maze() / .complexity_of_maze()
                                              (maze_complexity_evaluation.py:298-329)
  solution = astar_limited_partial(maze, start, goal)
  MetricsCalculator(maze, len(solution)).calculate_L / calculate_DE / calculate_D (solution)
                                              (metrics_calculator.py:11-133)

(The script itself imports a misspelled class name; the library methods are used.)
Test infrastructure only; the committed file is data. Regenerate:

    python tests/golden/make_golden_metrics.py [--ref /root/reference]
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

from make_golden import load_reference  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    a = ap.parse_args()
    R = load_reference(a.ref)
    import golden_io as G
    from lib.a_star_algos.a_star import astar_limited_partial
    from lib.maze_difficulty_evaluation.metrics_calculator import MetricsCalculator
    from lib.maze_difficulty_evaluation.maze_complexity_evaluation import ComplexityEvaluation
    out = {k: [] for k in ("idx", "L", "DE", "D", "AC", "FDE", "BDE", "difficulty", "complexity")}
    for i, m in enumerate(G.mazes("gen_euclid.npz")):
        grid = m["grid"].astype(int).tolist()
        sol = astar_limited_partial(grid, m["start"], m["goal"])
        mc = MetricsCalculator(grid, len(sol))
        ac, fde, bde = mc.calculate_DE_sub(sol)
        try:
            ce = ComplexityEvaluation(grid, m["start"], m["goal"])
            dif, cpx = float(ce.difficulty_of_maze()), float(ce.complexity_of_maze())
        except Exception:  # log(0) on degenerate tiny mazes
            dif = cpx = float("nan")
        out["idx"].append(i)
        out["L"].append(mc.calculate_L(sol))
        out["DE"].append(mc.calculate_DE(sol))
        out["D"].append(mc.calculate_D(sol))
        out["AC"].append(ac)
        out["FDE"].append(fde)
        out["BDE"].append(bde)
        out["difficulty"].append(dif)
        out["complexity"].append(cpx)
        print(i, G.ALGOS[m["algo"]], m["n"], m["seed"], out["L"][-1], out["DE"][-1], out["D"][-1],
              cpx, flush=True)
    np.savez_compressed(os.path.join(HERE, "metrics.npz"),
                        **{k: np.array(v, np.int32 if k == "idx" else np.float64) for k, v in out.items()})


if __name__ == "__main__":
    main()
