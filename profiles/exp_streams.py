#!/usr/bin/env python3
"""Env shards on concurrent HIP streams: S shards of B/S instances, each stepped on its own
stream (fused act + step + autoreset), launches interleaved. Prints the aggregate vector-step
time for the whole B, to compare with one launch over all B instances."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))

import torch  # noqa: E402

import mazerl  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=300)
    a = ap.parse_args()
    for S in (1, 2, 4):
        streams = [torch.cuda.Stream() for _ in range(S)]
        envs = []
        for i, st in enumerate(streams):
            with torch.cuda.stream(st):
                envs.append(mazerl.VectorMazeEnv(a.envs // S, 81, enrich=True, seed=0x5EED0000 + i * (a.envs // S),
                                                 window=True, window_bits=False, pos=False, done_list=False))
        torch.cuda.synchronize()

        def run(n, k0):
            for k in range(n):
                for env, st in zip(envs, streams):
                    with torch.cuda.stream(st):
                        env.step_act(eps=1.0, seed=7, counter=k0 + k, autoreset=True)
        run(20, 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(a.iters, 100)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.iters
        print(json.dumps({"shards": S, "envs": a.envs, "us_per_vector_step": round(dt * 1e6, 2),
                          "env_steps_per_s": a.envs / dt}), flush=True)
        for e in envs:
            e.close()
        del envs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
