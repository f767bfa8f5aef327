#!/usr/bin/env python
"""A/B timing of dd_policy_rollout builds (actor + sampling + frame per frame,
one launch), interleaved ABBA rounds; prints us per frame per variant.

    python tools/lab/prl_lab.py --variants base,lnchain --envs 65536 --compute f16x3
"""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "reinforcement-learning-101_amd"))
import torch  # noqa: E402
from torch import nn  # noqa: E402

from delivery_drone_amd import EnvConfig, MlpNet, VecDroneEnv, abi  # noqa: E402

LAB = os.path.join(REPO, "reinforcement-learning-101_amd", "delivery_drone_amd", "_native", "lab")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variants", default="base")
    p.add_argument("--envs", default="65536")
    p.add_argument("--frames", type=int, default=64)
    p.add_argument("--rounds", type=int, default=10)
    p.add_argument("--compute", default="f16x3")
    args = p.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = nn.Sequential(nn.Linear(15, 128), nn.LayerNorm(128), nn.ReLU(), nn.Linear(128, 128), nn.LayerNorm(128),
                        nn.ReLU(), nn.Linear(128, 64), nn.LayerNorm(64), nn.ReLU(), nn.Linear(64, 3))
    sd = net.state_dict()
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=0)
    for n in [int(x) for x in args.envs.split(",")]:
        runs = {}
        for v in args.variants.split(","):
            lib = abi.load(os.path.join(LAB, f"lib_{v}.so"))
            env = VecDroneEnv(n, device=dev, config=cfg, library=lib)
            env.reset()
            actor = MlpNet(sd, device=dev, compute=args.compute, library=lib)
            bufs = dict(obs_out=torch.empty(args.frames, n, 15, device=dev),
                        actions_out=torch.empty(args.frames, n, dtype=torch.uint8, device=dev),
                        log_prob_out=torch.empty(args.frames, n, device=dev),
                        reward_out=torch.empty(args.frames, n, device=dev),
                        done_out=torch.empty(args.frames, n, dtype=torch.bool, device=dev))
            env.policy_rollout(actor, args.frames, **bufs)
            runs[v] = (env, actor, bufs, [])
        torch.cuda.synchronize()
        names = list(runs)
        for rnd in range(args.rounds):
            for v in (names if rnd % 2 == 0 else names[::-1]):
                env, actor, bufs, times = runs[v]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                env.policy_rollout(actor, args.frames, step=rnd * args.frames, **bufs)
                e1.record()
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1) * 1e3 / args.frames)
        for v, (_, _, _, times) in runs.items():
            print(json.dumps({"envs": n, "frames": args.frames, "compute": args.compute, "variant": v,
                              "us_per_frame_median": round(statistics.median(times), 3),
                              "us_per_frame_min": round(min(times), 3)}), flush=True)
        del runs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
