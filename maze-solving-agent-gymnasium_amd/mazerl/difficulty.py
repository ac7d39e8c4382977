"""McClendon maze difficulty (maze_complexity_evaluation.py:38-329) via libmazerl's native
mz_difficulty — used by get_maze_difficulty and best-of-6 generation (base_maze_env.py:78-105)."""
import ctypes as C

import numpy as np

from . import _native as N


def maze_difficulty(grid, start, goal):
    """ComplexityEvaluation(grid, start, goal).difficulty_of_maze() for a euclidean grid."""
    g = np.ascontiguousarray(grid, dtype=np.uint8)
    out = C.c_double()
    N.check(N.load().mz_difficulty(g.ctypes.data, g.shape[0], g.shape[1], int(start[0]),
                                   int(start[1]), int(goal[0]), int(goal[1]), C.byref(out)))
    return out.value


def toroidal_difficulty(grid, start, goal):
    """Difficulty of a cropped toroidal maze, evaluated on its bordered (N+2) grid like
    gen_maze_no_border (maze_generation.py:49-51) and the trainer (off_policy_trainer.py:194-196)."""
    g = np.pad(np.asarray(grid, np.uint8), 1)
    return maze_difficulty(g, (start[0] + 1, start[1] + 1), (goal[0] + 1, goal[1] + 1))


def difficulty_batch(env, env_ids=None, complexity=False):
    """McClendon difficulty (and complexity) of resident mazes of a VectorMazeEnv, one GPU
    workgroup per maze (mz_difficulty_batch, csrc/mz_mcclendon.hip; a toroidal maze scored as its
    bordered maze, as the reference scores it); mazes the kernel leaves to the host (nonzero
    status: cycles, open border squares, very long hallways, ...) go through mz_difficulty.
    Returns float64 numpy [n] (or ([n], [n]) with complexity) — math.log of the kernel's
    product / sum, the C library's log as the reference's math.log."""
    import math

    import torch
    dev = env.device
    ids = None if env_ids is None else torch.as_tensor(env_ids, dtype=torch.int32, device=dev)
    n = env.num_envs if ids is None else int(ids.numel())
    out = torch.empty(max(n, 1), 2, dtype=torch.float64, device=dev)
    st = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    lib = N.load()
    rc = lib.mz_difficulty_batch(env._h, None if ids is None else ids.data_ptr(), n,
                                 out.data_ptr(), st.data_ptr(), env._stream())
    host_ids = ids.cpu().numpy() if ids is not None else np.arange(n, dtype=np.int32)
    if rc == -2:  # MZ_EINVAL_SHAPE: pitch beyond the kernel's LDS plan, all on the host
        pw, stat = np.zeros((n, 2)), np.full(n, 2, np.int32)
    else:
        N.check(rc)
        pw, stat = out[:n].cpu().numpy(), st[:n].cpu().numpy()  # .cpu() waits for the stream
    d = np.empty(n)
    c = np.empty(n)
    for i in range(n):
        if stat[i] == 0:
            d[i] = math.log(pw[i, 0])
            c[i] = math.log(pw[i, 1])
            continue
        e = int(host_ids[i])
        q = env.query(e)
        g = env.grid(e)
        s, t = (q["start_r"], q["start_c"]), (q["goal_r"], q["goal_c"])
        if env.toroidal:
            d[i] = toroidal_difficulty(g, s, t)
            c[i] = toroidal_complexity(g, s, t)
        else:
            d[i], c[i] = maze_complexity(g, s, t)
    return (d, c) if complexity else d


def screen_batch(env, env_ids=None):
    """The order-free McClendon screen of resident euclidean mazes (mz_screen_batch,
    csrc/mz_screen.hip: one wave per maze): (prod [n], bound [n], status [n]) numpy — the product
    whose log is the difficulty, summed in an order of its own, a rigorous bound on its relative
    distance from the reference's float64 evaluation, status 0 ok / 2 declined."""
    import torch
    dev = env.device
    ids = None if env_ids is None else torch.as_tensor(env_ids, dtype=torch.int32, device=dev)
    n = env.num_envs if ids is None else int(ids.numel())
    out = torch.zeros(max(n, 1), 2, dtype=torch.float64, device=dev)
    st = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)
    N.check(N.load().mz_screen_batch(env._h, None if ids is None else ids.data_ptr(), n,
                                     out.data_ptr(), st.data_ptr(), env._stream()))
    o = out[:n].cpu().numpy()
    return o[:, 0].copy(), o[:, 1].copy(), st[:n].cpu().numpy()


def maze_complexity(grid, start, goal):
    """(difficulty_of_maze(), complexity_of_maze()) of a euclidean grid (host, mz_maze_complexity)."""
    g = np.ascontiguousarray(grid, dtype=np.uint8)
    d, c = C.c_double(), C.c_double()
    N.check(N.load().mz_maze_complexity(g.ctypes.data, g.shape[0], g.shape[1], int(start[0]),
                                        int(start[1]), int(goal[0]), int(goal[1]),
                                        C.byref(d), C.byref(c)))
    return d.value, c.value


def toroidal_complexity(grid, start, goal):
    g = np.pad(np.asarray(grid, np.uint8), 1)
    return maze_complexity(g, (start[0] + 1, start[1] + 1), (goal[0] + 1, goal[1] + 1))[1]
