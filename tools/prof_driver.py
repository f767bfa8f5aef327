#!/usr/bin/env python
"""Minimal GPU driver for rocprofv3 passes: runs one kernel family a few
times so a PMC pass sees only it.  --what step|rollout|mlp."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "reinforcement-learning-101_amd"))
import torch  # noqa: E402
from delivery_drone_amd import EnvConfig, VecDroneEnv, abi  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--what", default="rollout")
    p.add_argument("--envs", type=int, default=65536)
    p.add_argument("--frames", type=int, default=256)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--lib", default="")
    p.add_argument("--compute", default="f32", help="mlp: f32 or f16x3")
    args = p.parse_args()
    dev = torch.device("cuda", 0)
    lib = abi.load(args.lib) if args.lib else None
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=0)
    n = args.envs
    kw = {"library": lib} if lib is not None else {}
    env = VecDroneEnv(n, device=dev, config=cfg, **kw)
    env.reset()
    if args.what == "rollout":
        acts = torch.randint(0, 8, (args.frames, n), device=dev, dtype=torch.uint8)
        obs = torch.empty(args.frames, n, 15, device=dev)
        rew = torch.empty(args.frames, n, device=dev)
        done = torch.empty(args.frames, n, device=dev, dtype=torch.bool)
        for _ in range(args.reps):
            env.rollout(acts, obs_out=obs, reward_out=rew, done_out=done)
    elif args.what == "mlp":
        from torch import nn
        from delivery_drone_amd import MlpNet
        torch.manual_seed(0)
        net = nn.Sequential(nn.Linear(15, 128), nn.LayerNorm(128), nn.ReLU(), nn.Linear(128, 128),
                            nn.LayerNorm(128), nn.ReLU(), nn.Linear(128, 64), nn.LayerNorm(64), nn.ReLU(),
                            nn.Linear(64, 3))
        kw2 = {"library": lib} if lib is not None else {}
        kw2["compute"] = args.compute
        actor = MlpNet(net.state_dict(), device=dev, **kw2)
        o = torch.randn(n, 15, device=dev)
        acts_out = torch.empty(n, dtype=torch.uint8, device=dev)
        lp = torch.empty(n, device=dev)
        for k in range(args.reps):
            actor.act(o, step=k, actions_out=acts_out, log_prob_out=lp)
    elif args.what == "prl":  # dd_policy_rollout: actor + sampling + frame, `frames` per launch
        from torch import nn
        from delivery_drone_amd import MlpNet
        torch.manual_seed(0)
        net = nn.Sequential(nn.Linear(15, 128), nn.LayerNorm(128), nn.ReLU(), nn.Linear(128, 128),
                            nn.LayerNorm(128), nn.ReLU(), nn.Linear(128, 64), nn.LayerNorm(64), nn.ReLU(),
                            nn.Linear(64, 3))
        kw2 = {"library": lib} if lib is not None else {}
        actor = MlpNet(net.state_dict(), device=dev, compute=args.compute, **kw2)
        frames = min(args.frames, 64)
        for k in range(args.reps):
            env.policy_rollout(actor, frames, step=k * frames)
    elif args.what == "step":
        rows = torch.randint(0, 8, (8, n), device=dev, dtype=torch.uint8)
        for k in range(args.reps):
            env.step(rows[k % 8])
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
