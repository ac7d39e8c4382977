#!/usr/bin/env python3
"""Learner GEMMs: f32 (hipBLASLt f32 MFMA) vs bf16x3 as ONE bf16 GEMM over a tripled K
([Ah | Ah | Al] . [Bh | Bl | Bh]^T = Ah Bh^T + Ah Bl^T + Al Bh^T, f32 accumulate, f32 out via
torch.mm(..., out_dtype=float32)). Shapes: the PPO minibatch (2,048 rows) and the DDQN update
(2,048 stacked rows) fc1 / fc2 forward, dX, dW. Prints one JSON line: us per GEMM (split passes
included / excluded) and the max relative error vs float64."""
import json
import sys

import os

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "maze-solving-agent-gymnasium_amd"))


def split3(x, dim):
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    return hi, lo


def cat_k(a, b, ka, kb):
    """operands with the reduction dim ka of a and kb of b tripled."""
    ah, al = split3(a, ka)
    bh, bl = split3(b, kb)
    return torch.cat((ah, ah, al), dim=ka), torch.cat((bh, bl, bh), dim=kb)


def timed(fn, iters=50):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / iters * 1e3, 2)


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    out = {}
    M = 2048
    for (K, N) in ((1574, 1024), (1024, 512)):
        x = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) * 0.03
        g = torch.randn(M, N, device=dev)
        cases = {
            "fwd": (x, w.t(), 1, 0),     # [M,K] . [K,N]
            "dX": (g, w, 1, 0),          # [M,N] . [N,K]
            "dW": (g.t(), x, 1, 0),      # [N,M] . [M,K]
        }
        for name, (a, b, ka, kb) in cases.items():
            ref = (a.double() @ b.double())
            f32 = lambda: a @ b
            y32 = f32()
            a3, b3 = cat_k(a, b, ka, kb)
            x3 = lambda: torch.mm(a3, b3, out_dtype=torch.float32)
            y3 = x3()
            x3full = lambda: torch.mm(*cat_k(a, b, ka, kb), out_dtype=torch.float32)
            from mazerl.agents.linear import mm_x3
            k3 = lambda: mm_x3(a, b.t())
            yk = k3()
            scale = ref.abs().max()
            flop = 2 * a.shape[0] * a.shape[1] * b.shape[1]
            t32, t3, t3f, tk = timed(f32), timed(x3), timed(x3full), timed(k3)
            out[f"{K}x{N}_{name}"] = {
                "f32_us": t32, "x3_gemm_us": t3, "x3_with_split_us": t3f,
                "f32_tflops": round(flop / t32 / 1e6, 1), "x3_gemm_tflops_f32eq": round(flop / t3 / 1e6, 1),
                "err_f32": float(((y32.double() - ref).abs().max() / scale)),
                "err_x3": float(((y3.double() - ref).abs().max() / scale)),
                "mz_gemm_x3_us": tk, "mz_gemm_x3_tflops_f32eq": round(flop / tk / 1e6, 1),
                "err_mz_gemm_x3": float(((yk.double() - ref).abs().max() / scale)),
            }
            print(name, K, N, out[f"{K}x{N}_{name}"], file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
