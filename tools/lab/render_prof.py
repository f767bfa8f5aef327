#!/usr/bin/env python
"""Driver for rocprofv3 passes over dd_render: `frames` lanes (default 64) of a
running batch per launch, HUD on, `reps` launches (no graph, so each dispatch
is its own trace record)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "reinforcement-learning-101_amd"))
import torch  # noqa: E402
from delivery_drone_amd import EnvConfig, VecDroneEnv  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device("cuda", 0)
env = VecDroneEnv(4096, device=dev, config=EnvConfig(randomize_drone=True, auto_reset=False, seed=0))
env.reset()
acts = torch.randint(0, 8, (4096,), device=dev, dtype=torch.uint8)
for _ in range(60):
    env.step(acts)
lanes = torch.arange(0, 4096, 4096 // frames, dtype=torch.int32, device=dev)[:frames]
out = torch.empty(frames, 600, 800, 3, dtype=torch.uint8, device=dev)
for _ in range(reps):
    env.render(lanes=lanes, out=out, actions=acts)
torch.cuda.synchronize()
