"""ctypes view of the CPU oracle (oracle/mzoracle.c). TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module — as the
checker, never as the thing measured or shipped. The product (libmazerl.so, package `mazerl`)
never imports it.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libmzoracle.so")


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


class _Env(C.Structure):
    _fields_ = [("H", C.c_int), ("W", C.c_int), ("toroidal", C.c_int), ("enrich", C.c_int),
                ("sr", C.c_int), ("sc", C.c_int), ("gr", C.c_int), ("gc", C.c_int),
                ("max_steps", C.c_int), ("astar_mode", C.c_int),
                ("grid", C.c_void_p), ("D", C.c_void_p), ("visits", C.c_void_p),
                ("nonvisited", C.c_void_p),
                ("r", C.c_int), ("c", C.c_int), ("steps", C.c_int), ("inv", C.c_int),
                ("nmoves", C.c_int), ("prev_r", C.c_int), ("prev_c", C.c_int)]


class Obs(C.Structure):
    _fields_ = [("reward", C.c_double), ("truncated", C.c_int), ("terminated", C.c_int),
                ("r", C.c_int), ("c", C.c_int), ("best_r", C.c_int), ("best_c", C.c_int),
                ("distance", C.c_double), ("window", C.c_uint8 * 675)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(
                os.path.getmtime(os.path.join(HERE, f)) for f in ("mzoracle.c", "mzpygen.c", "mzmetrics.c", "mzoracle.h")):
            build()
        L = C.CDLL(LIB)
        u8p, i32p = C.POINTER(C.c_uint8), C.POINTER(C.c_int32)
        ip = C.POINTER(C.c_int)
        L.mzo_bfs.argtypes = [u8p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, i32p]
        L.mzo_astar_len.argtypes = [u8p] + [C.c_int] * 8
        L.mzo_goal_select.argtypes = [u8p, C.c_int, C.c_int, C.c_int, C.c_int, ip, ip]
        L.mzo_max_steps.argtypes = [u8p] + [C.c_int] * 7
        L.mzo_generate.argtypes = [u8p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64,
                                   ip, ip, ip, ip]
        L.mzo_philox.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.POINTER(C.c_uint32)]
        u32p = C.POINTER(C.c_uint32)
        L.mzo_generate_py.argtypes = [u8p, C.c_int, C.c_int, C.c_int, u32p, ip, ip, ip, ip]
        L.mzo_mt_seed.argtypes = [C.c_uint64, u32p]
        L.mzo_mt_below.argtypes = [u32p, C.c_uint32]
        L.mzo_mt_below.restype = C.c_uint32
        L.mzo_tuple_hash.argtypes = [C.c_int, C.c_int]
        L.mzo_tuple_hash.restype = C.c_uint64
        L.mzo_metrics.argtypes = [u8p] + [C.c_int] * 6 + [C.POINTER(C.c_double)]
        L.mzo_env_init.argtypes = [C.POINTER(_Env), u8p] + [C.c_int] * 9
        L.mzo_env_free.argtypes = [C.POINTER(_Env)]
        L.mzo_env_reset.argtypes = [C.POINTER(_Env), C.POINTER(Obs)]
        L.mzo_env_step.argtypes = [C.POINTER(_Env), C.c_int, C.POINTER(Obs)]
        L.mzo_env_mask.argtypes = [C.POINTER(_Env), C.c_int, C.POINTER(C.c_float)]
        L.mzo_best_next.argtypes = [C.POINTER(_Env), C.c_int, C.c_int, ip, ip]
        L.mzo_bench.argtypes = [u8p] + [C.c_int] * 10 + [C.c_long, C.c_int, C.c_uint64,
                                                          C.POINTER(C.c_long)]
        L.mzo_bench.restype = C.c_double
        _lib = L
    return _lib


def _u8(a):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return a, a.ctypes.data_as(C.POINTER(C.c_uint8))


def bfs(grid, src, toroidal=False):
    g, gp = _u8(grid)
    H, W = g.shape
    d = np.empty((H, W), np.int32)
    lib().mzo_bfs(gp, H, W, int(toroidal), int(src[0]), int(src[1]),
                  d.ctypes.data_as(C.POINTER(C.c_int32)))
    return d


def astar_len(grid, src, goal, toroidal=False, max_depth=-1):
    g, gp = _u8(grid)
    H, W = g.shape
    return lib().mzo_astar_len(gp, H, W, int(toroidal), int(src[0]), int(src[1]), int(goal[0]),
                               int(goal[1]), int(max_depth))


def goal_select(grid, start):
    g, gp = _u8(grid)
    H, W = g.shape
    r, c = C.c_int(), C.c_int()
    rc = lib().mzo_goal_select(gp, H, W, int(start[0]), int(start[1]), C.byref(r), C.byref(c))
    return None if rc else (r.value, c.value)


def max_steps(grid, start, goal, toroidal=False):
    g, gp = _u8(grid)
    H, W = g.shape
    return lib().mzo_max_steps(gp, H, W, int(toroidal), int(start[0]), int(start[1]),
                               int(goal[0]), int(goal[1]))


def generate(n, algo, seed, toroidal=False):
    g = np.zeros((n, n), np.uint8)
    out = [C.c_int() for _ in range(4)]
    rc = lib().mzo_generate(g.ctypes.data_as(C.POINTER(C.c_uint8)), n, n, int(toroidal),
                            int(algo), C.c_uint64(seed), *[C.byref(o) for o in out])
    if rc:
        raise ValueError(f"mzo_generate failed rc={rc}")
    return (out[0].value, out[1].value), (out[2].value, out[3].value), g


def mt_state(seed):
    """random.seed(seed)'s MT19937 state as uint32[625] (624 words + index)."""
    st = np.zeros(625, np.uint32)
    lib().mzo_mt_seed(C.c_uint64(seed), st.ctypes.data_as(C.POINTER(C.c_uint32)))
    return st


def generate_py(n, algo, state, toroidal=False):
    """gen_maze((n,n), algo) (toroidal: gen_maze_no_border) as CPython runs it from the
    random state `state` (uint32[625], advanced in place; or an int seed)."""
    if not isinstance(state, np.ndarray):
        state = mt_state(int(state))
    g = np.zeros((n, n), np.uint8)
    out = [C.c_int() for _ in range(4)]
    rc = lib().mzo_generate_py(g.ctypes.data_as(C.POINTER(C.c_uint8)), n, int(toroidal), int(algo),
                               state.ctypes.data_as(C.POINTER(C.c_uint32)), *[C.byref(o) for o in out])
    if rc:
        raise ValueError(f"mzo_generate_py failed rc={rc}")
    return (out[0].value, out[1].value), (out[2].value, out[3].value), g


def metrics(grid, start, goal):
    """MetricsCalculator L, DE, D, AC, FDE, BDE of the solution path (euclidean, perfect maze)."""
    g, gp = _u8(grid)
    H, W = g.shape
    out = (C.c_double * 6)()
    rc = lib().mzo_metrics(gp, H, W, int(start[0]), int(start[1]), int(goal[0]), int(goal[1]), out)
    if rc:
        raise ValueError("goal unreachable")
    return list(out)


def philox(key, ctr_hi, ctr_lo):
    o = (C.c_uint32 * 4)()
    lib().mzo_philox(C.c_uint64(key), C.c_uint64(ctr_hi), C.c_uint64(ctr_lo), o)
    return list(o)


class Env:
    """Single-instance restated env; mirrors BaseMazeEnv.step/reset/get_mask_direction."""

    def __init__(self, grid, start, goal, toroidal=False, enrich=True, astar_mode=False):
        g, gp = _u8(grid)
        self.H, self.W = g.shape
        self._e = _Env()
        lib().mzo_env_init(C.byref(self._e), gp, self.H, self.W, int(toroidal), int(enrich),
                           int(start[0]), int(start[1]), int(goal[0]), int(goal[1]),
                           int(astar_mode))
        self._o = Obs()

    @property
    def max_steps(self):
        return self._e.max_steps

    def __del__(self):
        try:
            lib().mzo_env_free(C.byref(self._e))
        except Exception:
            pass

    def _out(self):
        o = self._o
        return dict(reward=o.reward, truncated=bool(o.truncated), terminated=bool(o.terminated),
                    pos=(o.r, o.c), best_dir=(o.best_r, o.best_c), distance=o.distance,
                    window=np.frombuffer(bytes(o.window), np.uint8).reshape(3, 15, 15).copy())

    def reset(self):
        lib().mzo_env_reset(C.byref(self._e), C.byref(self._o))
        return self._out()

    def step(self, a):
        lib().mzo_env_step(C.byref(self._e), int(a), C.byref(self._o))
        return self._out()

    def mask(self, probs):
        m = (C.c_float * 4)()
        lib().mzo_env_mask(C.byref(self._e), int(probs), m)
        return np.array(list(m), np.float32)

    def best_next(self, r, c):
        a, b = C.c_int(), C.c_int()
        lib().mzo_best_next(C.byref(self._e), int(r), int(c), C.byref(a), C.byref(b))
        return a.value, b.value


def bench(grid, start, goal, toroidal, enrich, astar_mode, nenv, steps_per_env, threads, seed=1):
    g, gp = _u8(grid)
    H, W = g.shape
    tot = C.c_long()
    secs = lib().mzo_bench(gp, H, W, int(toroidal), int(enrich), int(start[0]), int(start[1]),
                           int(goal[0]), int(goal[1]), int(astar_mode), int(nenv),
                           int(steps_per_env), int(threads), C.c_uint64(seed), C.byref(tot))
    return secs, tot.value
