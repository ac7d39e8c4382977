#!/usr/bin/env python3
"""Acting Q-head GEMM epilogues at 65,536 rows (bf16): fc2 1024->512 + ReLU as F.linear + relu_
vs torch._addmm_activation (hipBLASLt fused bias + ReLU epilogue); fc1 1600->1024 + LeakyReLU as
F.linear + leaky_relu_. HIP-event average per call, and the max |difference|."""
import json

import torch
import torch.nn.functional as F


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


n = 65536
bf = torch.bfloat16
h1 = torch.randn(n, 1024, device="cuda", dtype=bf)
w2 = torch.randn(512, 1024, device="cuda", dtype=bf) * 0.03
b2 = torch.randn(512, device="cuda", dtype=bf)
x = torch.randn(n, 1600, device="cuda", dtype=bf)
w1 = torch.randn(1024, 1600, device="cuda", dtype=bf) * 0.03
b1 = torch.randn(1024, device="cuda", dtype=bf)
ref = F.relu(F.linear(h1, w2, b2))
fused = torch._addmm_activation(b2, h1, w2.t())
res = {
    "fc2_linear_relu_us": timed(lambda: F.relu_(F.linear(h1, w2, b2))),
    "fc2_addmm_activation_us": timed(lambda: torch._addmm_activation(b2, h1, w2.t())),
    "fc2_linear_only_us": timed(lambda: F.linear(h1, w2, b2)),
    "fc1_linear_leaky_us": timed(lambda: F.leaky_relu_(F.linear(x, w1, b1), 0.01)),
    "fc1_linear_only_us": timed(lambda: F.linear(x, w1, b1)),
    "fc2_max_abs_diff": float((ref.float() - fused.float()).abs().max()),
}
print(json.dumps({k: round(v, 2) for k, v in res.items()}))
