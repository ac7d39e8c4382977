"""Loaders for the committed golden fixtures (tests/golden/*.npz; data only)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KIND_SIMPLE, KIND_ENRICH, KIND_TOR, KIND_TOR_ENRICH, KIND_VAR_ENRICH = 0, 1, 2, 3, 4
ALGOS = ["r-prim", "dfs", "prim&kill"]


def load(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def mazes(name):
    z = load(name)
    out = []
    for i in range(len(z["n"])):
        n = int(z["n"][i])
        out.append(dict(algo=int(z["algo"][i]), n=n, seed=int(z["seed"][i]),
                        grid=z["grid"][i, :n, :n].copy(), start=tuple(int(x) for x in z["start"][i]),
                        goal=tuple(int(x) for x in z["goal"][i]),
                        max_steps=int(z["max_steps"][i]), difficulty=float(z["difficulty"][i])))
    return out


def traces():
    z = load("traces.npz")
    out = []
    off = z["offsets"]
    for i in range(len(z["n"])):
        n = int(z["n"][i])
        s, e = int(off[i]), int(off[i + 1])
        t = dict(kind=int(z["kind"][i]), n=n, grid=z["grid"][i, :n, :n].copy(),
                 start=tuple(int(x) for x in z["start"][i]), goal=tuple(int(x) for x in z["goal"][i]),
                 max_steps=int(z["max_steps"][i]))
        for k in ("op", "mask_int", "mask_prob", "pos", "agent", "target", "best_dir", "reward",
                  "truncated", "terminated", "distance"):
            t[k] = z[k][s:e]
        w = np.unpackbits(z["window"][s:e], axis=1)[:, :675]
        t["window"] = w.reshape(-1, 3, 15, 15)
        t["toroidal"] = t["kind"] in (KIND_TOR, KIND_TOR_ENRICH)
        t["enrich"] = t["kind"] in (KIND_ENRICH, KIND_TOR_ENRICH, KIND_VAR_ENRICH)
        out.append(t)
    return out


def envs():
    """envs.npz: reference env constructors after random.seed(s) (make_golden_envs.py)."""
    z = load("envs.npz")
    kinds = [str(k) for k in z["kinds"]]
    out = []
    for i in range(len(z["n"])):
        n = int(z["n"][i])
        out.append(dict(kind=kinds[int(z["kind"][i])], ctor=int(z["ctor"][i]), algo=int(z["algo"][i]),
                        seed=int(z["seed"][i]), n=n, grid=z["grid"][i, :n, :n].copy(),
                        start=tuple(int(x) for x in z["start"][i]),
                        goal=tuple(int(x) for x in z["goal"][i]),
                        max_steps=int(z["max_steps"][i]), probe=int(z["probe"][i])))
    return out
