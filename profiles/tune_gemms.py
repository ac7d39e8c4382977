#!/usr/bin/env python3
"""GEMM solution tuning (PyTorch TunableOp over hipBLASLt / rocBLAS) for the learners' shapes, and
the timing of the acting forward and of one DDQN update with and without the tuned table.

  python profiles/tune_gemms.py measure            # default hipBLASLt heuristics
  python profiles/tune_gemms.py tune [out.csv]     # tune every GEMM shape below, write the table
  python profiles/tune_gemms.py measure tuned      # same timings reading the tuned table

Shapes: the acting Q-head (bf16, 65,536 rows: 1600->1024, 1024->512, 512->4) and the DDQN / PPO
updates (f32, 2,048 rows, forward and both backward GEMMs of 1574->1024->512->4 / ->1).
Measured on MI355X (r01g): default act 0.448 / DDQN update GEMMs 0.682 / PPO 0.905 ms; with the
tuned table 0.441 / 0.699 / 0.886 ms — within noise, so the product keeps hipBLASLt's heuristics
and ships no table."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))
import torch  # noqa: E402

TABLE = os.path.join(ROOT, "gpurun_out", "tunableop_results.csv")


def timed(fn, iters=30):
    for _ in range(5):
        fn()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def workloads(dev):
    from mazerl.agents.fused import FusedQ
    from mazerl.agents.nets import QNet
    from mazerl.agents.ppo import ActorCriticNet
    torch.manual_seed(0)
    n = 65536
    net = QNet(variant="ddqn").to(dev)
    fq = FusedQ(net, seed=1)
    g = torch.Generator(device=dev).manual_seed(0)
    bits = torch.randint(0, 2**31 - 1, (n, 22), generator=g, device=dev, dtype=torch.int32)
    obs6 = torch.rand(n, 6, generator=g, device=dev)
    b = 2048
    bb, ob = bits[:b].contiguous(), obs6[:b].contiguous()
    ac = ActorCriticNet(3, 6, 4, 32, 1024).to(dev)

    def act():
        with torch.no_grad():
            fq(obs6, bits)

    def qnet_fwd_bwd():
        net.zero_grad(set_to_none=True)
        net((ob, bb)).pow(2).sum().backward()
        with torch.no_grad():
            net((ob, bb))

    def ppo_fwd_bwd():
        ac.zero_grad(set_to_none=True)
        lo, v = ac((ob, bb))
        (lo.pow(2).sum() + v.pow(2).sum()).backward()

    return {"act": act, "qnet_update_gemms": qnet_fwd_bwd, "ppo_update_gemms": ppo_fwd_bwd}


def main():
    mode = sys.argv[1]
    dev = torch.device("cuda:0")
    if mode == "tune":
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(True)
        torch.cuda.tunable.set_max_tuning_duration(60)
        out = sys.argv[2] if len(sys.argv) > 2 else TABLE  # written when the process exits
        torch.cuda.tunable.set_filename(out, insert_device_ordinal=False)
        t0 = time.time()
        for name, fn in workloads(dev).items():
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            print(json.dumps({"tuned": name, "seconds": round(time.time() - t0, 1)}), flush=True)
        print(json.dumps({"table": out, "entries": len(torch.cuda.tunable.get_results())}))
        return
    if len(sys.argv) > 2 and sys.argv[2] == "tuned":
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(False)
        torch.cuda.tunable.set_filename(TABLE, insert_device_ordinal=False)
        torch.cuda.tunable.read_file(TABLE)
    out = {"mode": "tuned" if torch.cuda.tunable.is_enabled() else "default"}
    for name, fn in workloads(dev).items():
        out[name + "_ms"] = round(timed(fn), 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
