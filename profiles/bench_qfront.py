#!/usr/bin/env python3
"""Micro-benchmark of the fused acting stem (mz_q_front, csrc/mz_qnet.hip) at the headline
batch: 65,536 instances, with and without dropout. Prints one JSON line per mode with the
average launch time (HIP events on the launch stream) and the HBM rate of its algorithmic
bytes: 88 B window bits + 24 B obs6 read, 3,200 B bf16 feature row written per instance."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))

import torch  # noqa: E402

from mazerl import _native as N  # noqa: E402

ALG_BYTES = 88 + 24 + 3200


def main(n=65536, iters=200):
    L = N.load()
    g = torch.Generator().manual_seed(0)
    bits = torch.randint(0, 2**31, (n, 22), generator=g, dtype=torch.int64).to(torch.int32).cuda()
    obs6 = torch.randn(n, 6, generator=g).cuda()
    w = (torch.randn(32, 3, 3, 3, generator=g) * 0.3).cuda()
    b = (torch.randn(32, generator=g) * 0.1).cuda()
    out = torch.empty(n, 1600, dtype=torch.bfloat16, device="cuda")
    st = torch.cuda.current_stream()
    for p in (0.0, 0.2):
        def run(k):
            N.check(L.mz_q_front(bits.data_ptr(), obs6.data_ptr(), n, w.data_ptr(), b.data_ptr(), p,
                                 1, k, out.data_ptr(), 1600, st.cuda_stream))
        for k in range(10):
            run(k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for k in range(iters):
            run(k)
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        print(json.dumps({"kernel": "k_qfront", "n": n, "dropout": p, "avg_us": round(ms * 1e3, 2),
                          "alg_GBps": round(n * ALG_BYTES / (ms * 1e-3) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
