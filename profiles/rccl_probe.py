"""Probe: can RCCL ("nccl" backend) run N ranks on the one GPU of a gpurun box?
Usage: python profiles/rccl_probe.py <world> -> one JSON line per rank (result or error).
Each rank binds cuda:0, all-reduces a vector, and times a 8.56 MB all-reduce (the learner's bucket)."""
import json
import os
import socket
import sys
import time

import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    rec = {"rank": rank, "world": world}
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("nccl", init_method="env://", device_id=dev)
        x = torch.full((1024,), float(rank + 1), device=dev)
        dist.all_reduce(x)
        torch.cuda.synchronize()
        rec["allreduce_ok"] = bool((x == world * (world + 1) / 2).all())
        g = torch.randn(2140548, device=dev)
        for _ in range(5):
            dist.all_reduce(g)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            dist.all_reduce(g)
        torch.cuda.synchronize()
        rec["bucket_8.56MB_us"] = (time.perf_counter() - t0) / 20 * 1e6
        rec["backend"] = dist.get_backend()
        rec["rccl_version"] = ".".join(map(str, torch.cuda.nccl.version())) if hasattr(torch.cuda, "nccl") else None
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 - a probe records whatever fails
        rec["error"] = f"{type(e).__name__}: {e}"[:600]
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    mp.spawn(worker, args=(world, _port()), nprocs=world, join=True)
