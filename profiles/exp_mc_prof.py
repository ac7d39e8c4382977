#!/usr/bin/env python3
"""Round 5: one k_mcclendon launch over 6,000 81x81 candidates per algorithm (for rocprofv3 --pmc
passes; the library is chosen by MZ_LIB_OVERRIDE, e.g. an MZ_MC_PROBE variant). Prints the kernel
time (HIP events, 3 launches after a warm one) as one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))

import torch  # noqa: E402


def main():
    from mazerl import VectorMazeEnv
    from mazerl import _native as N
    dev = torch.device("cuda", 0)
    algos = sys.argv[1].split(",") if len(sys.argv) > 1 else ["r-prim", "dfs", "prim&kill"]
    rec = {"lib": os.environ.get("MZ_LIB_OVERRIDE", "default")}
    for algo in algos:
        env = VectorMazeEnv(6000, 81, enrich=True, device=dev, algorithm=algo, seed=0x7E57,
                            done_list=False, pos=False, window=False, window_bits=False)
        res = torch.empty(6000, 2, dtype=torch.float64, device=dev)
        st = torch.empty(6000, dtype=torch.int32, device=dev)
        lib, s = N.load(), env._stream()
        N.check(lib.mz_difficulty_batch(env._h, None, 6000, res.data_ptr(), st.data_ptr(), s))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            N.check(lib.mz_difficulty_batch(env._h, None, 6000, res.data_ptr(), st.data_ptr(), s))
        e1.record()
        torch.cuda.synchronize()
        rec[algo] = round(e0.elapsed_time(e1) / 3, 3)
        rec[algo + "_status_nonzero"] = int((st != 0).sum())
        env.close()
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
