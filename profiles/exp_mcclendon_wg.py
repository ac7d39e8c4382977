#!/usr/bin/env python3
"""Round 4: k_mcclendon workgroup size A/B (MZ_MC_T = 256 / 512 / 1024 threads per maze). The set-
order hallway pass runs one wave per hallway; with ~143 KB of LDS per maze one workgroup holds a
CU, so more waves per workgroup = more hallways in flight. Library chosen by MZ_LIB_OVERRIDE;
prints one JSON line: kernel ms per 6,000 81x81 candidates per algorithm (HIP events) and a
checksum of the {prod, sum} outputs (must not change with the workgroup size)."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))

import torch  # noqa: E402


def main():
    from mazerl import VectorMazeEnv
    from mazerl import _native as N
    from mazerl.trainers.vector_trainer import make_env
    dev = torch.device("cuda", 0)
    rec = {"lib": os.environ.get("MZ_LIB_OVERRIDE", "default")}
    h = hashlib.sha256()
    for tor in (False, True):
        for algo in ("r-prim", "dfs", "prim&kill"):
            if tor:
                env = make_env(3000, list(range(17, 80, 2)), toroidal=True, algorithm=algo,
                               seed=0x70E5, device=dev, done_list=False, pos=False, window=False,
                               window_bits=False)
            else:
                env = VectorMazeEnv(6000, 81, enrich=True, device=dev, algorithm=algo, seed=0x7E57,
                                    done_list=False, pos=False, window=False, window_bits=False)
            n = env.num_envs
            res = torch.empty(n, 2, dtype=torch.float64, device=dev)
            st = torch.empty(n, dtype=torch.int32, device=dev)
            lib, s = N.load(), env._stream()
            for _ in range(2):
                N.check(lib.mz_difficulty_batch(env._h, None, n, res.data_ptr(), st.data_ptr(), s))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                N.check(lib.mz_difficulty_batch(env._h, None, n, res.data_ptr(), st.data_ptr(), s))
            e1.record()
            torch.cuda.synchronize()
            rec[("tor_" if tor else "") + algo] = round(e0.elapsed_time(e1) / 5, 3)
            h.update(res.cpu().numpy().tobytes())
            h.update(st.cpu().numpy().tobytes())
            env.close()
    rec["checksum"] = h.hexdigest()[:16]
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
