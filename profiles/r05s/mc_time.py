#!/usr/bin/env python3
"""Round 5: where k_mcclendon's phase-G lane path spends its cycles (MZ_MC_PROBE = 80 library in
MZ_LIB_OVERRIDE). Per 81x81 algorithm (6,000 candidates): the lane path's passes (BFS, copy,
split points, merge, rebuild, edge terms) in cycles per lane wave (mean over the 12 lane waves,
then over mazes), and the longest lane wave / the longest wave of G2 per maze."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))

import torch  # noqa: E402


def main():
    from mazerl import VectorMazeEnv
    from mazerl import _native as N
    dev = torch.device("cuda", 0)
    for algo in ("r-prim", "dfs", "prim&kill"):
        env = VectorMazeEnv(6000, 81, enrich=True, device=dev, algorithm=algo, seed=0x7E57,
                            done_list=False, pos=False, window=False, window_bits=False)
        n = env.num_envs
        res = torch.empty(n, 2, dtype=torch.float64, device=dev)
        st = torch.empty(n, dtype=torch.int32, device=dev)
        lib, s = N.load(), env._stream()
        N.check(lib.mz_difficulty_batch(env._h, None, n, res.data_ptr(), st.data_ptr(), s))
        torch.cuda.synchronize()
        r = res.cpu().numpy().astype(np.uint64)
        t = st.cpu().numpy().astype(np.uint32)
        m17 = np.uint64(131071)
        p = [(r[:, 0] & m17), (r[:, 0] >> np.uint64(17)) & m17, (r[:, 0] >> np.uint64(34)) & m17,
             (r[:, 1] & m17), (r[:, 1] >> np.uint64(17)) & m17, (r[:, 1] >> np.uint64(34)) & m17]
        names = ["bfs", "copy", "split_points", "merge", "rebuild", "edge_terms"]
        rec = {"algo": algo, "pass_cycles_per_lane_wave": {k: round(float(v.mean()) * 16) for k, v in zip(names, p)},
               "max_lane_wave_cycles": round(float((t & 0xFFFF).mean()) * 64),
               "max_g2_wave_cycles": round(float((t >> 16).mean()) * 64)}
        print(json.dumps(rec), flush=True)
        env.close()


if __name__ == "__main__":
    main()
