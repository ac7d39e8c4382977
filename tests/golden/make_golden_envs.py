#!/usr/bin/env python3
"""Golden fixture envs.npz: the maze the reference's env constructors build after
random.seed(s) (best-of-6 by McClendon difficulty, base_maze_env.py:78-97 /
toroidal_maze_env.py:40-54, from the global `random` stream), plus a probe of the stream position
afterwards (random.getrandbits(32)) — so a drop-in env must consume the global stream draw for
draw like the reference.

Test infrastructure only (runs in the build container where /root/reference exists, with the
offline gymnasium/pygame stand-ins of _refstubs.py). The committed file is data. Regenerate:

    python tests/golden/make_golden_envs.py [--ref /root/reference]
"""
import argparse
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import load_reference  # noqa: E402

ALGOS = ["r-prim", "dfs", "prim&kill"]
# (class key, constructor size): fixed-size envs take the maze shape, variable ones the max shape
CASES = [("simple_enrich", 15), ("simple_enrich", 21), ("simple", 25), ("toroidal_enrich", 17),
         ("toroidal", 21), ("simple_variable", 23), ("toroidal_variable", 33)]


def build(R, key, n):
    sme, tme = R["sme"], R["tme"]
    import gymnasium_env.envs.toroidal_variable_maze_env as tvme
    cls = {"simple": sme.SimpleMazeEnv, "simple_enrich": sme.SimpleEnrichMazeEnv,
           "toroidal": tme.ToroidalMazeEnv, "toroidal_enrich": tme.ToroidalEnrichMazeEnv,
           "simple_variable": R["svme"].SimpleVariableMazeEnv,
           "toroidal_variable": tvme.ToroidalVariableMazeEnv}[key]
    return cls((n, n))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--seeds", type=int, default=3)
    a = ap.parse_args()
    R = load_reference(a.ref)
    from gymnasium_env.envs.base_maze_env import BaseMazeEnv
    rows = []
    for key, n in CASES:
        for algo in ALGOS:
            for s in range(a.seeds):
                BaseMazeEnv.ALGORITHM = algo
                random.seed(1000 + s)
                env = build(R, key, n)
                probe = random.getrandbits(32)
                grid = np.array(env.maze_map, np.uint8)
                rows.append((key, n, algo, 1000 + s, grid, tuple(env._start_pos),
                             tuple(int(x) for x in env._target_location), int(env.max_steps_taken),
                             probe))
                print(key, n, algo, s, grid.shape, probe, flush=True)
    maxn = max(r[4].shape[0] for r in rows)
    grids = np.zeros((len(rows), maxn, maxn), np.uint8)
    for i, r in enumerate(rows):
        grids[i, :r[4].shape[0], :r[4].shape[1]] = r[4]
    keys = sorted({r[0] for r in rows})
    np.savez_compressed(
        os.path.join(HERE, "envs.npz"),
        kinds=np.array(keys), kind=np.array([keys.index(r[0]) for r in rows], np.int8),
        ctor=np.array([r[1] for r in rows], np.int16),
        algo=np.array([ALGOS.index(r[2]) for r in rows], np.int8),
        seed=np.array([r[3] for r in rows], np.int32),
        n=np.array([r[4].shape[0] for r in rows], np.int16), grid=grids,
        start=np.array([r[5] for r in rows], np.int16), goal=np.array([r[6] for r in rows], np.int16),
        max_steps=np.array([r[7] for r in rows], np.int32),
        probe=np.array([r[8] for r in rows], np.uint32))


if __name__ == "__main__":
    main()
