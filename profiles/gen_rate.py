#!/usr/bin/env python3
"""Maze generation throughput on the GPU (k_build, one wave per maze): mazes/s for each
algorithm, Philox vs CPython-exact rng, at the headline 65,536 x 81x81 (and toroidal 41x41)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))

import torch  # noqa: E402

import mazerl  # noqa: E402


def main(B=65536):
    quick = "--philox-81" in sys.argv  # only the headline size's Philox builds
    for tor, dim in ((False, 81),) if quick else ((False, 81), (True, 41)):
        env = mazerl.VectorMazeEnv(B, dim, toroidal=tor, enrich=True, generate=False)
        for rng in ("philox",) if quick else ("philox", "cpython"):
            for algo in ("r-prim", "dfs", "prim&kill"):
                env.generate(algorithm=algo, seed=1, rng=rng)  # warm (LDS attr, code load)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                env.generate(algorithm=algo, seed=2, rng=rng)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                import hashlib
                h = hashlib.sha256(env.meta().cpu().numpy().tobytes()).hexdigest()[:12]
                print(json.dumps({"lib": os.path.basename(os.environ.get("MZ_LIB_OVERRIDE", "default")),
                                  "meta_hash": h, "grid": dim, "toroidal": tor, "rng": rng, "algo": algo,
                                  "mazes": B, "seconds": round(dt, 4),
                                  "mazes_per_s": round(B / dt)}), flush=True)
        env.close()


if __name__ == "__main__":
    main()
