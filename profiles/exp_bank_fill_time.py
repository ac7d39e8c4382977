#!/usr/bin/env python3
"""Maze-bank fill rate per algorithm: a fresh 4,096-instance 81x81 handle, enable_bank(slots=K) fills
both banks (2 K Philox r-prim builds through mz_bank_fill -> k_cand_build / k_cand_build_rprim),
timed with HIP events, for the library named by MZ_LIB_OVERRIDE; plus a hash of one bank's meta
words via bank_slot for a few slots (the same mazes either way)."""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))

import torch  # noqa: E402


def main(K=16384, reps=3):
    for algo in ("r-prim", "dfs", "prim&kill"):
        one(algo, K, reps)


def one(algo, K, reps):
    from mazerl import VectorMazeEnv
    dev = torch.device("cuda", 0)
    out = []
    for r in range(reps + 1):
        env = VectorMazeEnv(4096, 81, enrich=True, device=dev, algorithm=algo, seed=0xB0B0,
                            done_list=False, window=False, window_bits=True)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        env.enable_bank(slots=K, algorithms=[algo])
        e.record()
        torch.cuda.synchronize()
        if r:
            out.append(s.elapsed_time(e))
        if r == reps:
            h = hashlib.sha256()
            for slot in (0, 1, K // 2, K - 1):
                g, sg = env.bank_slot(0, algo, 81, slot)
                h.update(g.tobytes())
                h.update(repr(sg).encode())
        env.close()
    ms = min(out)
    print(json.dumps({"lib": os.path.basename(os.environ.get("MZ_LIB_OVERRIDE", "default")),
                      "algorithm": algo, "builds": 2 * K, "ms": ms, "mazes_per_s": 2 * K / ms * 1e3,
                      "slots_sha": h.hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()
