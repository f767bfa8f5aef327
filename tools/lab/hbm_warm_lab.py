#!/usr/bin/env python
"""Diagnostic: does the 16.8M-drone step (HBM-resident) speed up with
sustained load?  Times consecutive blocks of graph replays on one env and
prints each block's device time per step (HIP events), plus the same after
an idle pause."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "reinforcement-learning-101_amd"))
import torch  # noqa: E402
from delivery_drone_amd import EnvConfig, VecDroneEnv  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16_777_216
    blocks = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    dev = torch.device("cuda", 0)
    env = VecDroneEnv(n, device=dev, config=EnvConfig(randomize_drone=True, randomize_platform=True,
                                                       auto_reset=True, seed=0))
    env.reset()
    rows = torch.randint(0, 8, (4, n), device=dev, dtype=torch.uint8)
    stream = torch.cuda.Stream(dev)
    with torch.cuda.stream(stream):
        for k in range(3):
            env.step(rows[k % 4])
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for k in range(10):
                env.step(rows[k % 4])
    torch.cuda.synchronize()

    def block(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(stream):
            e0.record(stream)
            for _ in range(reps):
                g.replay()
            e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / (reps * 10)

    t0 = time.time()
    for b in range(blocks):
        us = block(10)
        print(json.dumps({"phase": "sustained", "block": b, "t_s": round(time.time() - t0, 3), "us_per_step": round(us, 2)}),
              flush=True)
    time.sleep(2.0)
    for b in range(4):
        us = block(10)
        print(json.dumps({"phase": "after_idle_2s", "block": b, "us_per_step": round(us, 2)}), flush=True)


if __name__ == "__main__":
    main()
