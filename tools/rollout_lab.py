#!/usr/bin/env python
"""A/B timing of dd_rollout builds (interleaved rounds, one process)."""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "reinforcement-learning-101_amd"))
import torch  # noqa: E402
from delivery_drone_amd import EnvConfig, VecDroneEnv, abi  # noqa: E402

LAB = os.path.join(REPO, "reinforcement-learning-101_amd", "delivery_drone_amd", "_native", "lab")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variants", default="base")
    p.add_argument("--envs", default="65536,262144")
    p.add_argument("--frames", type=int, default=256)
    p.add_argument("--rounds", type=int, default=7)
    p.add_argument("--no-obs", action="store_true")
    p.add_argument("--philox", action="store_true", help="in-kernel Philox actions (config 5b) instead of a tensor")
    p.add_argument("--warm", type=int, default=0, help="untimed back-to-back launches first (the DVFS steady state)")
    p.add_argument("--burst", type=int, default=1, help="back-to-back launches per variant and round, each timed")
    args = p.parse_args()
    dev = torch.device("cuda", 0)
    cfg = EnvConfig(randomize_drone=True, auto_reset=True, seed=0)
    for n in [int(x) for x in args.envs.split(",")]:
        acts = torch.randint(0, 8, (args.frames, n), device=dev, dtype=torch.uint8)
        obs = torch.empty(args.frames, n, 15, device=dev)
        rew = torch.empty(args.frames, n, device=dev)
        done = torch.empty(args.frames, n, device=dev, dtype=torch.bool)
        envs = {}
        shared = VecDroneEnv(n, device=dev, config=cfg)
        shared.reset()
        for v in args.variants.split(","):
            # every variant steps the same buffers (physical placement out of the A/B)
            e = VecDroneEnv.__new__(VecDroneEnv)
            e.__dict__.update(shared.__dict__)
            e._lib = abi.load(os.path.join(LAB, f"lib_{v}.so"), abi_versions=(11, 12))
            e.rollout(None if args.philox else acts, frames=args.frames, obs_out=obs, reward_out=rew, done_out=done,
                      write_obs=not args.no_obs)
            envs[v] = (e, [])
        torch.cuda.synchronize()
        names = list(envs)
        for _ in range(args.warm):
            for v in names:
                envs[v][0].rollout(None if args.philox else acts, frames=args.frames, obs_out=obs, reward_out=rew,
                                   done_out=done, write_obs=not args.no_obs)
        torch.cuda.synchronize()
        for rnd in range(args.rounds):  # ABBA: alternate the order so position effects cancel
            for v in (names if rnd % 2 == 0 else names[::-1]):
                e, ts = envs[v]
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                       for _ in range(args.burst)]
                for e0, e1 in evs:
                    e0.record()
                    e.rollout(None if args.philox else acts, frames=args.frames, obs_out=obs, reward_out=rew,
                              done_out=done, write_obs=not args.no_obs)
                    e1.record()
                torch.cuda.synchronize()
                ts.extend(e0.elapsed_time(e1) for e0, e1 in evs)
        for v, (e, ts) in envs.items():
            med = statistics.median(ts)
            print(json.dumps({"envs": n, "frames": args.frames, "variant": v, "obs": not args.no_obs, "philox": args.philox,
                              "ms_median": round(med, 4),
                              "steps_per_s": round(n * args.frames / (med * 1e-3), 1)}), flush=True)


if __name__ == "__main__":
    main()
