#!/usr/bin/env python
"""Eager config-3 steps from one lab build (for counter passes that want
plain launches: rocprofv3 --pmc over tools/lab/sq_step_ab.sh).

    python tools/lab/step_eager.py --variant base --envs 262144 --steps 40
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "reinforcement-learning-101_amd"))
import torch  # noqa: E402

from delivery_drone_amd import EnvConfig, VecDroneEnv, abi  # noqa: E402

LAB = os.path.join(REPO, "reinforcement-learning-101_amd", "delivery_drone_amd", "_native", "lab")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variant", default="base")
    p.add_argument("--envs", type=int, default=262_144)
    p.add_argument("--steps", type=int, default=40)
    p.add_argument("--warm", type=int, default=300)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    lib = abi.load(os.path.join(LAB, f"lib_{a.variant}.so"), abi_versions=(11, 12))
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=0)
    env = VecDroneEnv(a.envs, device=dev, config=cfg, library=lib)
    env.reset()
    g = torch.Generator(device=dev).manual_seed(1)
    rows = torch.randint(0, 8, (8, a.envs), device=dev, dtype=torch.uint8, generator=g)
    for t in range(a.warm + a.steps):  # the warm steps bring the batch to its steady mix of episodes
        env.step(rows[t % 8])
    torch.cuda.synchronize(dev)
    print(f"{a.variant}: {a.warm + a.steps} steps of {a.envs}")


if __name__ == "__main__":
    main()
