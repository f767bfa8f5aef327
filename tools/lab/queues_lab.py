#!/usr/bin/env python
"""Lab: one batch stepped as P lane ranges, each range its OWN hipGraph
replayed on its own stream (so on its own hardware queue), forked from and
joined to the timing stream once per replay.  concurrency_lab.py put the
ranges into one graph as parallel branches, and ROCm ran those branches one
after another; separate graphs on separate streams are what two processes
sharing a card do (profiles/r01/bench_g2_gloo_rehearsal.json: 1.3x).

variants: 'single' (one graph of the whole batch), 'qP' (P ranges, P graphs,
P streams), 'dP' (P whole batches of N drones each on P streams: the
two-process case inside one process; throughput is per P*N).
usage: queues_lab.py N gsteps variant [variant ...]
"""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "reinforcement-learning-101_amd"))
import torch  # noqa: E402
from delivery_drone_amd import EnvConfig, VecDroneEnv  # noqa: E402


def build(v, n, dev, cfg, rows, gsteps, streams):
    parts = 1 if v == "single" else int(v[1:])
    if v.startswith("d"):
        envs = [VecDroneEnv(n, device=dev, config=cfg, env_id_base=k * n) for k in range(parts)]
        ranges = [(e, None) for e in envs]
    else:
        env = VecDroneEnv(n, device=dev, config=cfg)
        envs = [env]
        ranges = [(env, slice(n * k // parts, n * (k + 1) // parts)) for k in range(parts)]
    for e in envs:
        e.reset()
    graphs = []
    for (e, sl), s in zip(ranges, streams):
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for j in range(3):
                r = rows[j % 4] if sl is None else rows[j % 4][sl]
                e.step(r, lanes=sl)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for j in range(gsteps):
                r = rows[j % 4] if sl is None else rows[j % 4][sl]
                e.step(r, lanes=sl)
        graphs.append(g)
    torch.cuda.synchronize()
    return parts if v.startswith("d") else 1, graphs


def main():
    dev = torch.device("cuda", 0)
    n = int(sys.argv[1])
    gsteps = int(sys.argv[2])
    variants = sys.argv[3:]
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=0)
    rows = torch.randint(0, 8, (4, n), device=dev, dtype=torch.uint8)
    s0 = torch.cuda.Stream(dev)
    side = [torch.cuda.Stream(dev) for _ in range(4)]
    runs = []
    for v in variants:
        mult, graphs = build(v, n, dev, cfg, rows, gsteps, side)
        runs.append((v, mult, graphs, []))
    for rnd in range(16):
        order = runs if rnd % 2 == 0 else list(reversed(runs))
        for v, mult, graphs, ts in order:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s0)
            for g, s in zip(graphs, side):
                s.wait_stream(s0)
                with torch.cuda.stream(s):
                    g.replay()
            for s in side[:len(graphs)]:
                s0.wait_stream(s)
            e1.record(s0)
            torch.cuda.synchronize()
            if rnd >= 2:
                ts.append(e0.elapsed_time(e1) * 1e3 / gsteps)
    for v, mult, graphs, ts in runs:
        med = statistics.median(ts)
        print(json.dumps({"n": n, "gsteps": gsteps, "variant": v, "us_per_step_median": round(med, 3),
                          "us_min": round(min(ts), 3),
                          "env_steps_per_s": round(mult * n / (med * 1e-6), 1)}), flush=True)


if __name__ == "__main__":
    main()
