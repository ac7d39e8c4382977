#!/usr/bin/env python3
"""fc1 weight-gradient GEMM of the DDQN update (dW = dY^T X: dY [2048, 1024], X [2048, 1574],
f32) in a few formulations: which one hipBLASLt serves fastest. HIP-event average per call."""
import json

import torch


def timed(fn, iters=50):
    for _ in range(5):
        fn()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


b, n_out, n_in = 2048, 1024, 1574
gy = torch.randn(b, n_out, device="cuda")
x = torch.randn(b, n_in, device="cuda")
w = torch.randn(n_out, n_in, device="cuda")
xp = torch.zeros(b, 1600, device="cuda")
xp[:, :n_in] = x
res = {
    "gyT_x": timed(lambda: gy.t() @ x),
    "xT_gy_T": timed(lambda: (x.t() @ gy).t()),
    "xT_gy_T_contig": timed(lambda: (x.t() @ gy).t().contiguous()),
    "gyT_x_pad1600": timed(lambda: gy.t() @ xp),
    "gy_w_dx": timed(lambda: gy @ w),
    "fwd_x_wT": timed(lambda: x @ w.t()),
    "fwd_xpad_wT": timed(lambda: xp @ torch.nn.functional.pad(w, (0, 26)).t()),
}
fl = 2.0 * b * n_out * n_in
print(json.dumps({k: {"us": round(v, 1), "tflops": round(fl / v / 1e6, 1)} for k, v in res.items()}))
