#!/usr/bin/env python3
"""Which layer's precision decides the acting argmax? (round 3, VERDICT "greedy acting precision")

Trains the bench's DDQN (bench.py win_rate setup, 2,400 vector steps), then on the newest 65,536
replay states (real trainer observations, dropout off) compares argmax of the f32 QNet with
emulated acting heads: each layer's input / weight rounded to bf16 (one MFMA) or split into a bf16
hi + lo pair with the three cross products summed in f32 ("bf16x3": hi*hi + hi*lo + lo*hi), the
products accumulated in f32 — what a bf16 MFMA kernel computes. Prints one JSON line.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def bf(x):
    return x.to(torch.bfloat16).to(torch.float32)


def split(x):
    hi = bf(x)
    return hi, bf(x - hi)


def lin(x, w, b, mode):
    """x @ w.T + b with operands in `mode`: f32 | bf16 | x3 (bf16 hi/lo, three products)."""
    if mode == "f32":
        return F.linear(x, w, b)
    if mode == "bf16":
        return F.linear(bf(x), bf(w)) + b
    xh, xl = split(x)
    wh, wl = split(w)
    return F.linear(xh, wh) + F.linear(xh, wl) + F.linear(xl, wh) + b


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--train-steps", type=int, default=2400)
    a = ap.parse_args()
    import bench
    args = bench.parse.__wrapped__() if hasattr(bench.parse, "__wrapped__") else None
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from mazerl import VectorMazeEnv
    from mazerl.agents.dqn import VectorDQNLearner
    from mazerl.trainers.vector_trainer import VectorOffPolicyTrainer
    B, dim = 65536, 81
    env = VectorMazeEnv(B, dim, enrich=True, device=dev, algorithm="r-prim", seed=0xA11CE,
                        done_list=False, window=False, window_bits=True)
    decay = ((dim - 1) * (dim - 1) // 2) * 5 / 40.0
    L = VectorDQNLearner(B, dev, variant="ddqn", lr=1e-3, eps_start=0.95, eps_final=0.1,
                         eps_decay=decay, gamma=0.7, batch_size=1024, capacity=2_000_000,
                         target_every=13, overlap=True, greedy_rows=True)
    tr = VectorOffPolicyTrainer(env, L, seed=3)
    tr.train(20)
    tr.train(a.train_steps)
    env.close()
    rp, n = L.replay, 65536
    idx = torch.arange(rp.ptr - n, rp.ptr, device=dev) % rp.capacity
    s6, sw = rp.s6.index_select(0, idx), rp.sw.index_select(0, idx)
    net = L.source
    net.eval()
    out = {}
    with torch.no_grad():
        from mazerl.agents.stem import stem_features
        feat = stem_features(sw, s6, net.conv[0], 0.0, None, 0)  # f32 [n, 1574]
        q32 = net((s6, sw))
        a32 = q32.argmax(1)
        fc = [m for m in net.fc if isinstance(m, torch.nn.Linear)]
        acts = [m for m in net.fc if not isinstance(m, torch.nn.Linear)]
        # the stem's own bf16 error: conv weight rounded (the window is exact)
        conv = net.conv[0]
        wsave = conv.weight.data.clone()
        conv.weight.data = bf(wsave)
        feat_bfw = stem_features(sw, s6, conv, 0.0, None, 0)
        conv.weight.data = wsave
        variants = {
            "all_bf16": ("bf16w", "bf16", "bf16", "bf16"),
            "all_x3": ("f32", "x3", "x3", "x3"),
            "stem_bf16w_fc_x3": ("bf16w", "x3", "x3", "x3"),
            "fc1_x3_rest_bf16": ("f32", "x3", "bf16", "bf16"),
            "fc1_fc2_x3_fc3_f32": ("f32", "x3", "x3", "f32"),
            "fc1_bf16_rest_x3": ("f32", "bf16", "x3", "x3"),
            "stem_f32_fc1_bf16_fc2_bf16_fc3_f32": ("f32", "bf16", "bf16", "f32"),
            "fc1_x3_fc2_bf16_fc3_f32": ("f32", "x3", "bf16", "f32"),
        }
        for name, (stem, m1, m2, m3) in variants.items():
            h = feat_bfw if stem == "bf16w" else feat
            h = acts[0](lin(h, fc[0].weight, fc[0].bias, m1))
            h = acts[1](lin(h, fc[1].weight, fc[1].bias, m2))
            q = lin(h, fc[2].weight, fc[2].bias, m3)
            err = ((q - q32).abs().amax(1) / q32.abs().amax(1).clamp_min(1e-30))
            out[name] = {"agreement": float((q.argmax(1) == a32).float().mean()),
                         "max_rel_err": float(err.max()), "mean_rel_err": float(err.mean())}
        # the product path: FusedQ (bf16 stem + hipBLASLt bf16 GEMMs)
        fused = L.fused
        fused.invalidate()
        qa = fused(s6, sw).float()
        out["fused_q_product"] = {"agreement": float((qa.argmax(1) == a32).float().mean())}
        top2 = q32.topk(2, dim=1).values
        gap = (top2[:, 0] - top2[:, 1]) / q32.abs().amax(1).clamp_min(1e-30)
        out["gap_quantiles"] = {str(p): float(gap.quantile(p)) for p in (0.001, 0.01, 0.05, 0.1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
