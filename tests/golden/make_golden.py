#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the reference's own Python code.

Test infrastructure only: runs in the build container (where /root/reference exists), never on
the GPU box, never imported by the product. The committed .npz files are DATA (inputs + expected
outputs); no reference source is copied. Regenerate with:

    python tests/golden/make_golden.py [--ref /root/reference]

What is captured (SURVEY.md §8c "golden vectors to commit"):
  gen_euclid.npz   gen_maze((N,N), algo) after random.seed(s)              lib/maze_generation.py:6-35
                   + max_steps (set_max_steps)                              simple_maze_env.py:52-58
                   + McClendon difficulty                                   maze_complexity_evaluation.py:319
  gen_toroid.npz   gen_maze_no_border((N,N), algo) after random.seed(s)     lib/maze_generation.py:37-56
                   + toroidal max_steps                                     toroidal_maze_env.py:71-77
  traces.npz       op-by-op env traces (step/reset) on those mazes: per op the pre-op direction
                   masks (probs False/True), and the post-op obs / reward / truncated /
                   terminated / info / window bits                          base_maze_env.py:136-210
"""
import argparse
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def load_reference(ref):
    import torch  # noqa: F401  (torch first, then stubs — SURVEY §8c recipe)
    sys.path.insert(0, HERE)
    import _refstubs
    _refstubs.install()
    sys.dont_write_bytecode = True
    sys.path.insert(0, ref)
    import lib.maze_generation as mg
    import lib.a_star_algos.a_star as astar
    import lib.a_star_algos.a_star_tor as astar_tor
    from lib.maze_difficulty_evaluation.metrics_calculator import MetricsCalculator
    from lib.maze_difficulty_evaluation.maze_complexity_evaluation import ComplexityEvaluation
    from gymnasium_env.envs import simple_maze_env, toroidal_maze_env, simple_variable_maze_env
    return dict(mg=mg, astar=astar, astar_tor=astar_tor, MC=MetricsCalculator,
                CE=ComplexityEvaluation, sme=simple_maze_env, tme=toroidal_maze_env,
                svme=simple_variable_maze_env)


def max_steps_of(R, grid, start, goal, toroidal):
    """Restates set_max_steps with the reference's own A*/MetricsCalculator objects."""
    import math
    fn = R["astar_tor"].astar_limited_partial if toroidal else R["astar"].astar_limited_partial
    path = fn(grid, start, tuple(goal))
    factor = R["MC"](grid, len(path)).calculate_L(path)
    h, w = len(grid), len(grid[0])
    return math.ceil((((h - 1) * (w - 1)) - 1) * factor)


def difficulty_of(R, grid, start, goal):
    try:
        return float(R["CE"](grid, start, goal).difficulty_of_maze())
    except Exception:  # log(0) etc. on degenerate tiny mazes
        return float("nan")


ALGOS = ["r-prim", "dfs", "prim&kill"]


def gen_euclid(R, sizes, seeds):
    rows = []
    for algo in ALGOS:
        for n in sizes:
            for s in seeds:
                random.seed(s)
                start, goal, grid = R["mg"].gen_maze((n, n), algo)
                ms = max_steps_of(R, grid, start, goal, False)
                dif = difficulty_of(R, grid, start, goal) if n <= 41 else float("nan")
                rows.append((algo, n, s, np.array(grid, np.uint8), start, goal, ms, dif))
    return rows


def gen_toroid(R, sizes, seeds):
    rows = []
    for algo in ALGOS:
        for n in sizes:
            for s in seeds:
                random.seed(s)
                start, goal, grid, dif = R["mg"].gen_maze_no_border((n, n), algo)
                ms = max_steps_of(R, grid, start, goal, True)
                rows.append((algo, n, s, np.array(grid, np.uint8), start, goal, ms, float(dif)))
    return rows


def pack_rows(rows, path):
    maxn = max(r[1] for r in rows)
    k = len(rows)
    grids = np.zeros((k, maxn, maxn), np.uint8)
    for i, r in enumerate(rows):
        grids[i, :r[1], :r[1]] = r[3]
    np.savez_compressed(
        path,
        algo=np.array([ALGOS.index(r[0]) for r in rows], np.int8),
        n=np.array([r[1] for r in rows], np.int16),
        seed=np.array([r[2] for r in rows], np.int32),
        grid=grids,
        start=np.array([r[4] for r in rows], np.int16),
        goal=np.array([r[5] for r in rows], np.int16),
        max_steps=np.array([r[6] for r in rows], np.int32),
        difficulty=np.array([r[7] for r in rows], np.float64),
    )


# ---------------------------------------------------------------------------------------------
# traces
# ---------------------------------------------------------------------------------------------
KIND_SIMPLE, KIND_ENRICH, KIND_TOR, KIND_TOR_ENRICH, KIND_VAR_ENRICH = 0, 1, 2, 3, 4


def make_env(R, kind, grid, start, goal):
    grid = [list(map(int, row)) for row in grid]
    start = (int(start[0]), int(start[1]))
    goal = (int(goal[0]), int(goal[1]))
    n = len(grid)
    fixed = lambda self, shape: (start, goal, [row[:] for row in grid])  # noqa: E731
    if kind in (KIND_SIMPLE, KIND_ENRICH):
        base = R["sme"].SimpleMazeEnv if kind == KIND_SIMPLE else R["sme"].SimpleEnrichMazeEnv
        cls = type("FixedEnv", (base,), {"generate_maze": fixed})
        return cls((n, n))
    if kind in (KIND_TOR, KIND_TOR_ENRICH):
        base = R["tme"].ToroidalMazeEnv if kind == KIND_TOR else R["tme"].ToroidalEnrichMazeEnv
        cls = type("FixedEnv", (base,), {"generate_maze": fixed})
        return cls((n, n))
    if kind == KIND_VAR_ENRICH:
        base = R["svme"].SimpleEnrichVariableMazeEnv
        cls = type("FixedEnv", (base,), {"generate_maze": fixed})
        env = cls((n + 8, n + 8))
        assert tuple(env.maze_shape) == (15, 15) and n == 15
        return env
    raise ValueError(kind)


DELTAS = [(1, 0), (-1, 0), (0, 1), (0, -1)]


def run_trace(R, kind, grid, start, goal, n_ops, rng):
    env = make_env(R, kind, grid, start, goal)
    enrich = kind in (KIND_ENRICH, KIND_TOR_ENRICH, KIND_VAR_ENRICH)
    rec = {k: [] for k in ("op", "mask_int", "mask_prob", "agent", "target", "best_dir", "reward",
                           "truncated", "terminated", "distance", "window", "pos")}
    obs, info = env.reset()
    # phase schedule: a wall-hammer phase (invalid-move counter past 250) and a ping-pong phase
    # (visit counts past 188) inside an otherwise mixed policy.
    hammer_at = int(rng.integers(50, 150))
    pingpong_at = hammer_at + 300
    t = 0
    pp_dir = None
    while t < n_ops:
        mi = np.asarray(env.get_mask_direction(probs=False)).astype(np.int32)
        mp = np.asarray(env.get_mask_direction(probs=True)).astype(np.float32)
        done_prev = rec["terminated"][-1] or rec["truncated"][-1] if rec["op"] else False
        if done_prev and rng.random() < 0.5 and not (hammer_at <= t < pingpong_at + 420):
            op = 4
        elif hammer_at <= t < hammer_at + 270:
            walls = np.flatnonzero(mi == 0)
            op = int(walls[0]) if len(walls) else int(rng.integers(4))
        elif pingpong_at <= t < pingpong_at + 420:
            if pp_dir is None:
                opens = np.flatnonzero(mi != 0)
                pp_dir = int(opens[0])
                op = pp_dir
            else:
                op = pp_dir ^ 1 if (t - pingpong_at) % 2 == 1 else pp_dir
        else:
            u = rng.random()
            greedy = t >= pingpong_at + 420  # final phase: mostly follow "best dir" -> wins
            if u < (0.1 if greedy else 0.55):
                p = mp / mp.sum()
                op = int(rng.choice(4, p=p))
            elif u < (0.97 if greedy else 0.85):
                bd = tuple(int(x) for x in np.asarray(obs["best dir"]))
                if bd == (0, 0):
                    op = int(rng.integers(4))
                else:
                    # best dir = agent - best_next  ->  move by -bd (euclidean); for wrapped
                    # toroidal values fall back to the sign
                    d = (-int(np.sign(bd[0])), -int(np.sign(bd[1])))
                    if abs(bd[0]) > 1 or abs(bd[1]) > 1:
                        d = (int(np.sign(bd[0])), int(np.sign(bd[1])))
                    op = DELTAS.index(d) if d in DELTAS else int(rng.integers(4))
            else:
                op = int(rng.integers(4))
        if op == 4:
            obs, info = env.reset()
            r, tr, te = 0.0, False, False
        else:
            obs, r, tr, te, info = env.step(op)
        rec["op"].append(op)
        rec["mask_int"].append(mi)
        rec["mask_prob"].append(mp)
        rec["pos"].append(np.array(env._agent_location, np.int64))
        rec["agent"].append(np.asarray(obs["agent"], np.float64))
        rec["target"].append(np.asarray(obs["target"], np.float64))
        rec["best_dir"].append(np.asarray(obs["best dir"], np.int64))
        rec["reward"].append(float(r))
        rec["truncated"].append(bool(tr))
        rec["terminated"].append(bool(te))
        rec["distance"].append(float(info["distance"]))
        if enrich:
            w = obs["window"].numpy()
            assert w.shape == (3, 15, 15), w.shape
            assert set(np.unique(w)).issubset({0.0, 1.0})
            rec["window"].append(np.packbits(w.reshape(-1).astype(np.uint8)))
        else:
            rec["window"].append(np.zeros(85, np.uint8))
        t += 1
    return rec, env.max_steps_taken


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--quick", action="store_true")
    args = ap.parse_args()
    R = load_reference(args.ref)

    seeds = list(range(8))
    print("euclidean generation ...", flush=True)
    ge = gen_euclid(R, [9, 15, 21, 41, 81], seeds if not args.quick else seeds[:2])
    pack_rows(ge, os.path.join(HERE, "gen_euclid.npz"))
    print("toroidal generation ...", flush=True)
    gt = gen_toroid(R, [9, 17, 21, 29, 41], seeds if not args.quick else seeds[:2])
    pack_rows(gt, os.path.join(HERE, "gen_toroid.npz"))

    print("traces ...", flush=True)
    cases = []
    # (kind, source rows, n, how many)
    plan = [(KIND_SIMPLE, ge, 9, 2), (KIND_ENRICH, ge, 15, 2), (KIND_VAR_ENRICH, ge, 15, 1),
            (KIND_ENRICH, ge, 21, 2), (KIND_ENRICH, ge, 41, 2), (KIND_ENRICH, ge, 81, 2),
            (KIND_TOR, gt, 9, 2), (KIND_TOR_ENRICH, gt, 9, 1), (KIND_TOR_ENRICH, gt, 17, 2),
            (KIND_TOR_ENRICH, gt, 21, 1), (KIND_TOR_ENRICH, gt, 29, 2), (KIND_TOR_ENRICH, gt, 41, 1)]
    rng = np.random.default_rng(1234)
    for kind, rows, n, cnt in plan:
        pool = [r for r in rows if r[1] == n]
        picks = rng.choice(len(pool), size=cnt, replace=False)
        for p in picks:
            algo, n_, s, grid, start, goal, ms, dif = pool[int(p)]
            rec, ms_env = run_trace(R, kind, grid, start, goal, 1500 if not args.quick else 200, rng)
            assert ms_env == ms, (ms_env, ms)
            cases.append((kind, n_, grid, start, goal, ms, rec))
            print(f"  kind={kind} n={n_} algo={algo} seed={s} max_steps={ms} "
                  f"wins={sum(rec['terminated'])} truncs={sum(rec['truncated'])}", flush=True)

    T = [len(c[6]["op"]) for c in cases]
    off = np.concatenate([[0], np.cumsum(T)]).astype(np.int64)
    maxn = max(c[1] for c in cases)
    grids = np.zeros((len(cases), maxn, maxn), np.uint8)
    for i, c in enumerate(cases):
        grids[i, :c[1], :c[1]] = c[2]
    cat = lambda k, dt: np.concatenate([np.asarray(c[6][k], dt) for c in cases])  # noqa: E731
    np.savez_compressed(
        os.path.join(HERE, "traces.npz"),
        kind=np.array([c[0] for c in cases], np.int8),
        n=np.array([c[1] for c in cases], np.int16),
        grid=grids,
        start=np.array([c[3] for c in cases], np.int16),
        goal=np.array([c[4] for c in cases], np.int16),
        max_steps=np.array([c[5] for c in cases], np.int32),
        offsets=off,
        op=cat("op", np.int8),
        mask_int=cat("mask_int", np.int8),
        mask_prob=cat("mask_prob", np.float32),
        pos=cat("pos", np.int16),
        agent=cat("agent", np.float64),
        target=cat("target", np.float64),
        best_dir=cat("best_dir", np.int16),
        reward=cat("reward", np.float64),
        truncated=cat("truncated", np.bool_),
        terminated=cat("terminated", np.bool_),
        distance=cat("distance", np.float64),
        window=cat("window", np.uint8),
    )
    print("done:", len(cases), "traces,", int(off[-1]), "ops")


if __name__ == "__main__":
    main()
