#!/usr/bin/env python
"""Placement diagnostic with counters: three identical 16.8M-drone envs,
each stepped in eager launches in a fixed order (env 0 x S, env 1 x S,
env 2 x S, twice), so a rocprofv3 --pmc / --kernel-trace run of this script
can attribute every step_kernel dispatch to its allocation by dispatch order.
Prints one JSON line per env with its own event timing (median us/step).

    rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum ... -- python3 tools/lab/placement_pmc.py [S]
"""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "reinforcement-learning-101_amd"))
import torch  # noqa: E402

from delivery_drone_amd import EnvConfig, VecDroneEnv  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 16_777_216
    dev = torch.device("cuda", 0)
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=0)
    rows = torch.randint(0, 8, (4, n), device=dev, dtype=torch.uint8)
    envs = []
    for _ in range(3):
        e = VecDroneEnv(n, device=dev, config=cfg)
        e.reset()
        envs.append(e)
    torch.cuda.synchronize()
    times = {k: [] for k in range(3)}
    for rnd in range(2):
        for k in range(3):
            for j in range(steps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                envs[k].step(rows[j % 4])
                e1.record()
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) * 1e3)
    for k in range(3):
        print(json.dumps({"env": k, "steps": len(times[k]), "us_median": round(statistics.median(times[k]), 1),
                          "x_ptr": hex(envs[k].x.data_ptr()), "obs_ptr": hex(envs[k].obs.data_ptr()),
                          "order": "env0 x S, env1 x S, env2 x S, twice"}), flush=True)


if __name__ == "__main__":
    main()
