#!/usr/bin/env python3
"""Decomposition of the headline vector step (65,536 x 81x81 r-prim Enrich) on the GPU:
k_step with each output set (f32 window, window bits only, no window), k_reset_done alone, and
the host-side cost of the Python/ctypes launch path. Prints one JSON line per measurement.

  python profiles/exp_kstep.py [--envs 65536] [--dim 81]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))

import torch  # noqa: E402

import mazerl  # noqa: E402
from mazerl import _build  # noqa: E402


def timed(fn, iters, st):
    for k in range(10):
        fn(k)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(st)
    for k in range(iters):
        fn(10 + k)
    e1.record(st)
    host = (time.perf_counter() - t0) / iters
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / iters
    return e0.elapsed_time(e1) / iters * 1e3, host * 1e6, wall * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--dim", type=int, default=81)
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--lib", default=None, help="alternative libmazerl build (A/B runs)")
    ap.add_argument("--modes", default="f32_window,bits_only,both,no_window")
    a = ap.parse_args()
    if a.lib:
        _build.LIB = os.path.abspath(a.lib)
    st = torch.cuda.current_stream()
    modes = [("f32_window", dict(window=True, window_bits=False)),
             ("bits_only", dict(window=False, window_bits=True)),
             ("both", dict(window=True, window_bits=True)),
             ("no_window", dict(window=False, window_bits=False))]
    for name, kw in modes:
        if name not in a.modes.split(","):
            continue
        env = mazerl.VectorMazeEnv(a.envs, a.dim, enrich=True, device="cuda:0", seed=0x5EED0000,
                                   pos=False, done_list=False, **kw)
        us, host, wall = timed(lambda k: env.step_act(eps=1.0, seed=7, counter=k), a.iters, st)
        print(json.dumps({"what": "k_step", "mode": name, "gpu_us": round(us, 2),
                          "host_us_per_call": round(host, 2), "wall_us": round(wall, 2)}), flush=True)
        if name == "f32_window" and not a.lib:
            us, host, wall = timed(lambda k: env.reset_done(), a.iters, st)
            print(json.dumps({"what": "k_reset_done", "gpu_us": round(us, 2),
                              "host_us_per_call": round(host, 2), "wall_us": round(wall, 2)}), flush=True)

            def vstep(k):
                env.step_act(eps=1.0, seed=7, counter=k)
                env.reset_done()
            us, host, wall = timed(vstep, a.iters, st)
            print(json.dumps({"what": "step+reset", "gpu_us": round(us, 2),
                              "host_us_per_call": round(host, 2), "wall_us": round(wall, 2)}), flush=True)
            us, host, wall = timed(lambda k: env.step_act(eps=1.0, seed=7, counter=k, autoreset=True),
                                   a.iters, st)
            print(json.dumps({"what": "step_autoreset", "gpu_us": round(us, 2),
                              "host_us_per_call": round(host, 2), "wall_us": round(wall, 2)}), flush=True)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(a.iters + 10)]

            def vstep_ev(k):
                evs[k][0].record(st)
                env.step_act(eps=1.0, seed=7, counter=k)
                evs[k][1].record(st)
                env.reset_done()
            us, host, wall = timed(vstep_ev, a.iters, st)
            ks = sum(evs[k][0].elapsed_time(evs[k][1]) for k in range(10, a.iters + 10)) / a.iters
            print(json.dumps({"what": "step+reset+events", "gpu_us": round(us, 2), "k_step_ev_us": round(ks * 1e3, 2),
                              "host_us_per_call": round(host, 2), "wall_us": round(wall, 2)}), flush=True)
        env.close()
        del env
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
