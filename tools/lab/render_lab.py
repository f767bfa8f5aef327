#!/usr/bin/env python
"""Timing of dd_render: `frames` lanes of a running 4,096-lane batch per launch
(HUD on or off; lanes that are done get the game-over overlay).  20 launches
captured in a hipGraph, replayed and timed with HIP events, so the number is
device time, not the Python wrapper's.

    --variants base,nolicm   A/B of lab builds (tools/build_variants.sh):
                             HUD and overlay on, 64 and 256 lanes, interleaved
                             rounds, median per variant."""
import argparse
import json
import statistics
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "reinforcement-learning-101_amd"))
import torch  # noqa: E402
from delivery_drone_amd import EnvConfig, VecDroneEnv, abi  # noqa: E402

LAB = os.path.join(REPO, "reinforcement-learning-101_amd", "delivery_drone_amd", "_native", "lab")


def ab(env, acts, variants, dev, rounds=9, reps=20):
    stream = torch.cuda.Stream(dev)
    libs = {v: abi.load(os.path.join(LAB, f"lib_{v}.so")) for v in variants}
    own = env._lib
    for frames in (64, 256):
        lanes = torch.arange(0, 4096, 4096 // frames, dtype=torch.int32, device=dev)[:frames]
        out = torch.empty(frames, 600, 800, 3, dtype=torch.uint8, device=dev)
        graphs, ts = {}, {v: [] for v in variants}
        with torch.cuda.stream(stream):
            for v in variants:
                env._lib = libs[v]
                env.render(lanes=lanes, out=out, actions=acts)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=stream):
                    for _ in range(reps):
                        env.render(lanes=lanes, out=out, actions=acts)
                graphs[v] = g
            for r in range(rounds):
                for v in (variants if r % 2 == 0 else variants[::-1]):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    graphs[v].replay()
                    e1.record(stream)
                    torch.cuda.synchronize()
                    ts[v].append(e0.elapsed_time(e1) * 1e3 / reps)
        for v in variants:
            print(json.dumps({"frames": frames, "variant": v, "us_median": round(statistics.median(ts[v]), 2),
                              "us_min": round(min(ts[v]), 2)}), flush=True)
    env._lib = own


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variants", default="")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    env = VecDroneEnv(4096, device=dev, config=EnvConfig(randomize_drone=True, auto_reset=False, seed=0))
    env.reset()
    acts = torch.randint(0, 8, (4096,), device=dev, dtype=torch.uint8)
    for _ in range(60):
        env.step(acts)
    if a.variants:
        ab(env, acts, a.variants.split(","), dev)
        return
    stream = torch.cuda.Stream(dev)
    for frames in (1, 16, 64, 256):
        lanes = torch.arange(0, 4096, 4096 // frames, dtype=torch.int32, device=dev)[:frames]
        out = torch.empty(frames, 600, 800, 3, dtype=torch.uint8, device=dev)
        for hud, over in ((True, True), (False, True), (False, False)):
            with torch.cuda.stream(stream):
                env.render(lanes=lanes, out=out, hud=hud, game_over=over, actions=acts)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                reps = 20
                with torch.cuda.graph(g, stream=stream):
                    for _ in range(reps):
                        env.render(lanes=lanes, out=out, hud=hud, game_over=over, actions=acts)
                g.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                g.replay()
                e1.record(stream)
                torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            gbs = frames * 1.44e6 / (us * 1e-6) / 1e9
            print(json.dumps({"frames": frames, "hud": hud, "game_over": over, "us": round(us, 2), "frames_per_s": round(frames / us * 1e6),
                              "gbs": round(gbs, 1), "done_lanes": int(env.done[lanes.long()].sum())}), flush=True)


if __name__ == "__main__":
    main()
