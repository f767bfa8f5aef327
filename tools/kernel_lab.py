#!/usr/bin/env python
"""A/B timing of step-kernel builds, interleaved in one process.

Each variant is a library under _native/lab/: lib_base.so (a copy of the
working tree's build) or a committed revision built by tools/build_rev.sh.  For every batch size, every variant gets its own
VecDroneEnv (config-3 workload: random spawn, auto-reset, obs on), a captured
hipGraph of G steps, and R interleaved rounds of replays timed with HIP events
on the replay stream.  Prints one JSON line per (N, variant): median and min
us/step and the algorithmic GB/s of the median.

    python tools/kernel_lab.py --variants base,ocml --envs 262144,16777216
"""
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
    p.add_argument("--envs", default="262144,16777216")
    p.add_argument("--graph-steps", type=int, default=20)
    p.add_argument("--rounds", type=int, default=9)
    p.add_argument("--precision", default="f32")
    p.add_argument("--no-obs", action="store_true")
    p.add_argument("--allocs", type=int, default=1,
                   help="identical envs allocated one after another; every variant steps each of them "
                        "(the HBM point's placement spread, DESIGN.md §4, then shows per allocation)")
    p.add_argument("--separate", dest="shared", action="store_false",
                   help="one env per variant (default: every variant steps the same buffers)")
    args = p.parse_args()
    dev = torch.device("cuda", 0)
    libs = {v: abi.load(os.path.join(LAB, f"lib_{v}.so"), abi_versions=(11, 12)) for v in args.variants.split(",")}
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=0)
    G = args.graph_steps
    for n in [int(x) for x in args.envs.split(",")]:
        rows = torch.randint(0, 8, (8, n), device=dev, dtype=torch.uint8)
        stream = torch.cuda.Stream(dev)
        runs = {}
        allocs = []
        for a in range(max(1, args.allocs)):
            shared = None
            for name, lib in libs.items():
                if shared is None or not args.shared:
                    env = VecDroneEnv(n, device=dev, config=cfg, precision=args.precision, library=lib)
                    env.reset()
                    shared = env
                    allocs.append(env)
                else:  # the same buffers, another build: physical placement out of the A/B
                    env = shared
                env._lib = lib
                with torch.cuda.stream(stream):
                    for k in range(3):
                        env.step(rows[k], write_obs=not args.no_obs)
                    torch.cuda.synchronize(dev)
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=stream):
                        for k in range(G):
                            env.step(rows[k % 8], write_obs=not args.no_obs)
                    g.replay()
                torch.cuda.synchronize(dev)
                runs[(name, a)] = (env, g, [])
        keys = list(runs)
        for rnd in range(args.rounds):  # ABBA: alternate the order so position effects cancel
            for key in (keys if rnd % 2 == 0 else keys[::-1]):
                env, g, times = runs[key]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                with torch.cuda.stream(stream):
                    e0.record(stream)
                    g.replay()
                    e1.record(stream)
                torch.cuda.synchronize(dev)
                times.append(e0.elapsed_time(e1) * 1e3 / G)
        for (name, a), (env, g, times) in runs.items():
            med = statistics.median(times)
            bpe = env.step_bytes_per_env(with_obs=not args.no_obs)
            row = {"envs": n, "variant": name, "us_per_step_median": round(med, 3),
                   "us_per_step_min": round(min(times), 3),
                   "gbs_median": round(bpe * n / (med * 1e-6) / 1e9, 1),
                   "steps_per_s": round(n / (med * 1e-6), 1)}
            if args.allocs > 1:
                row["allocation"] = a
            print(json.dumps(row), flush=True)
        del runs, allocs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
