#!/usr/bin/env python3
"""Best-of-6 bank fill rate (the trainers' refill work, base_maze_env.py:78-97 per win): a fresh
4,096-instance 81x81 handle, enable_bank(slots=K, candidates=6) fills both banks (2 K selections
of 6 candidates each), timed with HIP events, for the library named by MZ_LIB_OVERRIDE; a hash of
a few slots (the same mazes for every library) and the selection counters."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))

import torch  # noqa: E402


def one(algo, K, reps):
    from mazerl import VectorMazeEnv
    dev = torch.device("cuda", 0)
    out = []
    for r in range(reps + 1):
        env = VectorMazeEnv(4096, 81, enrich=True, device=dev, algorithm=algo, seed=0xB0B0,
                            done_list=False, window=False, window_bits=True)
        env.select_stats(reset=True)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        env.enable_bank(slots=K, algorithms=[algo], candidates=6)
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
            st = env.select_stats()
        env.close()
    ms = min(out)
    print(json.dumps({"lib": os.path.basename(os.environ.get("MZ_LIB_OVERRIDE", "default")),
                      "algorithm": algo, "selections": 2 * K, "candidates": 12 * K, "ms": round(ms, 3),
                      "selections_per_s": round(2 * K / ms * 1e3), "slots_sha": h.hexdigest()[:16],
                      "stats": st}), flush=True)


if __name__ == "__main__":
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    for algo in ("r-prim", "dfs", "prim&kill"):
        one(algo, K, 2)
