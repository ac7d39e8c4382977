#!/usr/bin/env python3
"""mz_colsum_f32 alone at the learner's bias-gradient shapes ([2,048 x 1,024], [2,048 x 512], the
head's [128 x 2,052] partials, [512 x 1,024] for config 4): HIP events over 500 launches, for the
library named by MZ_LIB_OVERRIDE. One JSON line per shape, with the max abs difference from a
float64 column sum."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))

import torch  # noqa: E402

from mazerl import _native as N  # noqa: E402


def main(iters=500):
    L = N.load()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    st = torch.cuda.current_stream(dev).cuda_stream
    for n, m in ((2048, 1024), (2048, 512), (128, 2052), (512, 1024)):
        x = torch.randn(n, m, device=dev, generator=g)
        out = torch.empty(m, device=dev)
        for _ in range(20):
            N.check(L.mz_colsum_f32(x.data_ptr(), n, m, m, out.data_ptr(), st))
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            L.mz_colsum_f32(x.data_ptr(), n, m, m, out.data_ptr(), st)
        e.record()
        torch.cuda.synchronize()
        err = (out.double() - x.double().sum(0)).abs().max().item()
        print(json.dumps({"lib": os.path.basename(os.environ.get("MZ_LIB_OVERRIDE", "default")),
                          "n": n, "m": m, "us_per_launch": s.elapsed_time(e) * 1e3 / iters,
                          "max_abs_err": err}), flush=True)


if __name__ == "__main__":
    main()
