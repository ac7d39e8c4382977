"""Drop-in for the reference's generator functions (lib/maze_generation.py:6-56).

gen_maze(shape, algorithm)            -> (start_point, goal_point, maze)
gen_maze_no_border(shape, algorithm)  -> (start_point, goal_point, maze, difficulty)

Both draw from Python's global `random` exactly as the reference does (start with
randrange(1, N - 1, 2) twice, then the algorithm's choices — CPython's MT19937 stream and set
iteration order emulated on the GPU, mz_generate_state), so `random.seed(s); gen_maze(...)` returns
the reference's own maze and leaves the global stream where the reference leaves it. The goal
(find_random_position :187-218: the dead end farthest from the start, first in row-major order
on ties) and the BFS that replaces its A* calls run on the GPU too; gen_maze_no_border's
McClendon difficulty is evaluated on the bordered maze before the crop (:47-51), in libmazerl's
native restatement (mz_difficulty).

Square shapes only (every reference caller passes one). An even size raises
IndexError like the reference (Q4: find_random_position indexes past the last row), but before
any draw is consumed. Algorithms: "dfs" (the reference's default), "r-prim", "prim&kill".
"""
import numpy as np

from ..difficulty import toroidal_difficulty
from ..vector_env import ALGOS, VectorMazeEnv

_envs = {}  # (dim, bordered) -> a 1-instance handle, reused across calls


def _handle(dim, toroidal):
    key = (dim, toroidal)
    env = _envs.get(key)
    if env is None:
        env = VectorMazeEnv(1, dim, toroidal=toroidal, enrich=False, generate=False, pos=False,
                            done_list=False)
        _envs[key] = env
    return env


def _check(shape, algorithm):
    rows, cols = int(shape[0]), int(shape[1])
    if rows != cols:
        raise ValueError(f"square mazes only (got {rows}x{cols})")
    if algorithm not in ALGOS:
        raise ValueError(f"unknown algorithm {algorithm!r}")
    return rows


def _grid(env):
    q = env.query(0)
    g = env.grid(0)
    return (q["start_r"], q["start_c"]), (q["goal_r"], q["goal_c"]), g


def gen_maze(shape, algorithm="dfs"):
    """maze_generation.py:6-35: (start_point, goal_point, maze) with maze a list of lists
    (0 wall, 1 floor, 2 goal) of size shape[0] x shape[0]."""
    n = _check(shape, algorithm)
    if n % 2 == 0:
        raise IndexError("list index out of range (even maze size, as the reference: SURVEY Q4)")
    env = _handle(n, False)
    env.generate_from_random(0, algorithm, dim=n)
    start, goal, g = _grid(env)
    return start, goal, g.astype(int).tolist()


def gen_maze_no_border(shape, algorithm="dfs"):
    """maze_generation.py:37-56: a (N+2) maze from gen_maze, its difficulty on the bordered maze,
    then the border cropped: (start_point, goal_point, maze, difficulty), coordinates shifted."""
    n = _check(shape, algorithm)
    if (n + 2) % 2 == 0:
        raise IndexError("list index out of range (even maze size, as the reference: SURVEY Q4)")
    env = _handle(n, True)  # the toroidal handle generates (N+2) and crops (gen_maze_no_border)
    env.generate_from_random(0, algorithm, dim=n)
    start, goal, g = _grid(env)
    difficulty = toroidal_difficulty(np.asarray(g, np.uint8), start, goal)
    return start, goal, g.astype(int).tolist(), difficulty
