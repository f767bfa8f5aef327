#!/usr/bin/env python
"""Lab: one batch stepped as P lane ranges on P streams captured as parallel
hipGraph branches.  Does a second kernel in flight hide one kernel's
dispatch ramp and its load -> compute -> store phases?

variants: 'single' (one dd_step per step), 'jP' (P ranges, joined every step),
'fP' (P ranges, forked once per graph and joined at its end: the ranges drift).
usage: concurrency_lab.py N variant [variant ...]
"""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "reinforcement-learning-101_amd"))
import torch  # noqa: E402
from delivery_drone_amd import EnvConfig, VecDroneEnv  # noqa: E402


def capture(env, rows, variant, gsteps, s0, side):
    n = env.num_envs
    g = torch.cuda.CUDAGraph()
    if variant == "single":
        parts = 1
    else:
        parts = int(variant[1:])
    bounds = [(n * k // parts, n * (k + 1) // parts) for k in range(parts)]
    streams = [s0] + side[:parts - 1]
    with torch.cuda.graph(g, stream=s0):
        if variant == "single":
            for j in range(gsteps):
                env.step(rows[j % 4])
        elif variant[0] == "j":
            for j in range(gsteps):
                for s in streams[1:]:
                    s.wait_stream(s0)
                for (a, b), s in zip(bounds, streams):
                    with torch.cuda.stream(s):
                        env.step(rows[j % 4][a:b], lanes=slice(a, b))
                for s in streams[1:]:
                    s0.wait_stream(s)
        else:
            for s in streams[1:]:
                s.wait_stream(s0)
            for j in range(gsteps):
                for (a, b), s in zip(bounds, streams):
                    with torch.cuda.stream(s):
                        env.step(rows[j % 4][a:b], lanes=slice(a, b))
            for s in streams[1:]:
                s0.wait_stream(s)
    return g


def main():
    dev = torch.device("cuda", 0)
    n = int(sys.argv[1])
    variants = sys.argv[2:]
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=0)
    rows = torch.randint(0, 8, (4, n), device=dev, dtype=torch.uint8)
    s0 = torch.cuda.Stream(dev)
    side = [torch.cuda.Stream(dev) for _ in range(7)]
    gsteps = 50
    runs = []
    for v in variants:
        env = VecDroneEnv(n, device=dev, config=cfg)
        env.reset()
        with torch.cuda.stream(s0):
            for j in range(3):
                env.step(rows[j % 4])
        torch.cuda.synchronize()
        runs.append((v, env, capture(env, rows, v, gsteps, s0, side), []))
    torch.cuda.synchronize()
    for rnd in range(14):
        order = runs if rnd % 2 == 0 else list(reversed(runs))
        for v, env, g, ts in order:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s0):
                e0.record(s0)
                g.replay()
                e1.record(s0)
            torch.cuda.synchronize()
            if rnd >= 2:
                ts.append(e0.elapsed_time(e1) * 1e3 / gsteps)
    for v, env, g, ts in runs:
        print(json.dumps({"n": n, "variant": v, "us_median": round(statistics.median(ts), 3),
                          "us_min": round(min(ts), 3)}), flush=True)


if __name__ == "__main__":
    main()
