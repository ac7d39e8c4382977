#!/usr/bin/env python3
"""fc1's input gradient in the DDQN update (dX = dY W: dY [2,048 x 1,024], W [1,024 x 1,574],
f32) in three layouts hipBLASLt may tile differently: NN as torch's autograd issues it, NT with
a transposed copy of W, and the transposed product dX^T = W^T dY^T made contiguous. HIP-event
average per call (including the copies each variant needs); one JSON line."""
import json

import torch


def timed(fn, iters=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / iters * 1e3, 1)


g = torch.Generator(device="cuda").manual_seed(0)
gy = torch.randn(2048, 1024, device="cuda", generator=g)
w = torch.randn(1024, 1574, device="cuda", generator=g) * 0.03
out = torch.empty(2048, 1574, device="cuda")
ref = gy @ w
res = {
    "nn_us": timed(lambda: torch.mm(gy, w, out=out)),
    "nt_with_wT_copy_us": timed(lambda: torch.mm(gy, w.t().contiguous().t(), out=out)),
    "nt_wT_cached_us": (lambda wt: timed(lambda: torch.mm(gy, wt.t(), out=out)))(w.t().contiguous()),
    "transposed_product_us": timed(lambda: out.copy_(torch.mm(w.t(), gy.t()).t())),
    "transposed_product_gemm_only_us": timed(lambda: torch.mm(w.t(), gy.t())),
}
res["max_abs_diff_transposed"] = float((torch.mm(w.t(), gy.t()).t() - ref).abs().max())
print(json.dumps(res), flush=True)
