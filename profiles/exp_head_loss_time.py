#!/usr/bin/env python3
"""mz_head_loss and mz_head_loss_backward alone (DDQN, stacked source rows, hidden 512) at update
batches 512 / 2,048 / 8,192: HIP events over 500 launches each, for the library named by
MZ_LIB_OVERRIDE (A/B builds). Prints one JSON line per batch with the loss bits and a hash of
diff, dz2 and the dW3 / db3 partials (kernel rewrites must keep them bit for bit)."""
import hashlib
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
    H = 512
    for b in (512, 2048, 8192):
        z2s = torch.randn(2 * b, H, device=dev, generator=g)
        z2t = torch.randn(b, H, device=dev, generator=g)
        w3s = torch.randn(4, H, device=dev, generator=g) * 0.05
        w3t = torch.randn(4, H, device=dev, generator=g) * 0.05
        b3s = torch.randn(4, device=dev, generator=g)
        b3t = torch.randn(4, device=dev, generator=g)
        act = torch.randint(0, 4, (b,), device=dev, generator=g)
        rew = torch.randn(b, device=dev, generator=g)
        part = torch.empty(max(1, L.mz_head_loss_workspace_floats(b)), device=dev)
        tk = torch.zeros(1, dtype=torch.int32, device=dev)
        loss = torch.empty((), device=dev)
        diff = torch.empty(b, device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream

        def launch():
            N.check(L.mz_head_loss(z2s.data_ptr(), H, w3s.data_ptr(), b3s.data_ptr(), z2t.data_ptr(),
                                   H, w3t.data_ptr(), b3t.data_ptr(), H, 1, 1, act.data_ptr(),
                                   rew.data_ptr(), 0.99, b, part.data_ptr(), tk.data_ptr(),
                                   loss.data_ptr(), diff.data_ptr(), st))
        gone = torch.ones((), device=dev)
        dz2 = torch.empty(2 * b, H, device=dev)
        nblk = L.mz_head_loss_backward_workspace_floats(b, H) // (4 * H + 4)
        bpart = torch.empty(nblk, 4 * H + 4, device=dev)

        def launch_bwd():
            N.check(L.mz_head_loss_backward(gone.data_ptr(), diff.data_ptr(), act.data_ptr(), b,
                                            z2s.data_ptr(), H, w3s.data_ptr(), H, 1, dz2.data_ptr(),
                                            H, bpart.data_ptr(), st))
        for _ in range(20):
            launch()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            launch()
        e.record()
        torch.cuda.synchronize()
        fwd_us = s.elapsed_time(e) * 1e3 / iters
        for _ in range(20):
            launch_bwd()
        torch.cuda.synchronize()
        s.record()
        for _ in range(iters):
            launch_bwd()
        e.record()
        torch.cuda.synchronize()
        h = hashlib.sha256()
        for t in (diff, dz2[:b], bpart):
            h.update(t.cpu().numpy().tobytes())
        print(json.dumps({"lib": os.path.basename(os.environ.get("MZ_LIB_OVERRIDE", "default")),
                          "b": b, "blocks": L.mz_head_loss_workspace_floats(b),
                          "us_per_launch": fwd_us, "bwd_us_per_launch": s.elapsed_time(e) * 1e3 / iters,
                          "out_sha": h.hexdigest()[:16],
                          "loss_bits": hex(int(loss.view(torch.int32).item()) & 0xFFFFFFFF),
                          "tickets_zero": bool((tk == 0).all().item())}), flush=True)


if __name__ == "__main__":
    main()
