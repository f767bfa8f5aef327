#!/usr/bin/env python
"""Lab: does the step's speed depend on where the SoA fields sit relative to
each other?  Every variant is its own env; 'torch' keeps the caching
allocator's placement, 'sS' carves all fields and outputs from one slab with
field k at a 2 MiB boundary + k*S bytes (tools/lab/diag_alloc.rebind_slab).
Timed in interleaved rounds (order reversed every other round).

usage: placement_lab.py N variant [variant ...]   e.g. 16777216 torch s0 s4096
"""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "reinforcement-learning-101_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import torch  # noqa: E402
from delivery_drone_amd import EnvConfig, VecDroneEnv  # noqa: E402
from diag_alloc import rebind_slab  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n = int(sys.argv[1])
    variants = sys.argv[2:]
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=0)
    rows = torch.randint(0, 8, (4, n), device=dev, dtype=torch.uint8)
    stream = torch.cuda.Stream(dev)
    gsteps = 10 if n > 4_000_000 else 50
    runs = []
    for v in variants:
        env = VecDroneEnv(n, device=dev, config=cfg)
        env.reset()
        if v != "torch":
            rebind_slab(env, int(v[1:]))
            torch.cuda.empty_cache()
        with torch.cuda.stream(stream):
            for j in range(3):
                env.step(rows[j % 4])
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                for j in range(gsteps):
                    env.step(rows[j % 4])
        runs.append((v, env, g, []))
    torch.cuda.synchronize()
    for rnd in range(12):
        order = runs if rnd % 2 == 0 else list(reversed(runs))
        for v, env, g, ts in order:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(stream):
                e0.record(stream)
                g.replay()
                e1.record(stream)
            torch.cuda.synchronize()
            if rnd >= 2:
                ts.append(e0.elapsed_time(e1) * 1e3 / gsteps)
    for v, env, g, ts in runs:
        offs = [(getattr(env, f).data_ptr() - env.x.data_ptr()) for f in ("y", "vx", "obs", "reward")]
        print(json.dumps({"n": n, "variant": v, "us_median": round(statistics.median(ts), 3),
                          "us_min": round(min(ts), 3), "x_ptr": hex(env.x.data_ptr()),
                          "offs_vs_x": offs}), flush=True)


if __name__ == "__main__":
    main()
