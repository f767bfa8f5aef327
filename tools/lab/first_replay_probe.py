#!/usr/bin/env python
"""Wall clock of a hipGraph of K config-3 steps on its FIRST replay (bench.py
times its K = 20 graph the first time it runs) against a replay of a graph
that has run before, and against a first replay after hipGraphUpload:

  fresh         a newly captured graph, timed on its first replay
  fresh_upload  a newly captured graph, hipGraphUpload'ed (and the stream
                synced) before its first, timed, replay
  warm          the same graph again (its second and later replays)

Each repetition: 5 warm-up steps from another graph, device sync, the timed
replay, device sync; perf_counter around it.  One JSON line per (K, method).

    python tools/lab/first_replay_probe.py --ks 20,50 --reps 15
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "reinforcement-learning-101_amd"), os.path.dirname(os.path.abspath(__file__))]

import torch  # noqa: E402
from span_events import KernelSpanEvents  # noqa: E402  (its handle on the HIP runtime torch loaded)

from delivery_drone_amd import EnvConfig, VecDroneEnv  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=262144)
    p.add_argument("--ks", default="20,50")
    p.add_argument("--reps", type=int, default=15)
    args = p.parse_args()
    dev = torch.device("cuda", 0)
    n = args.envs
    env = VecDroneEnv(n, device=dev, config=EnvConfig(randomize_drone=True, randomize_platform=True,
                                                      auto_reset=True, seed=0))
    env.reset()
    rows = torch.randint(0, 8, (8, n), device=dev, dtype=torch.uint8)
    stream = torch.cuda.Stream(dev)
    stream.wait_stream(torch.cuda.current_stream(dev))
    hip = KernelSpanEvents().hip
    sh = ctypes.c_void_p(stream.cuda_stream)
    with torch.cuda.stream(stream):
        for k in range(3):
            env.step(rows[k % 8])
        torch.cuda.synchronize(dev)

        def capture(k):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                for i in range(k):
                    env.step(rows[i % 8])
            return g

        warm5 = capture(5)
        warm5.replay()
        for k in [int(x) for x in args.ks.split(",")]:
            res = {"fresh": [], "fresh_upload": [], "warm": []}
            keep = capture(k)
            keep.replay()
            for rep in range(args.reps):
                for m in ("fresh", "fresh_upload", "warm"):
                    g = keep if m == "warm" else capture(k)
                    if m == "fresh_upload":
                        rc = hip.hipGraphUpload(ctypes.c_void_p(g.raw_cuda_graph_exec()), sh)
                        if rc != 0:
                            raise RuntimeError(f"hipGraphUpload: hipError {rc}")
                    warm5.replay()
                    torch.cuda.synchronize(dev)
                    t0 = time.perf_counter()
                    g.replay()
                    torch.cuda.synchronize(dev)
                    res[m].append((time.perf_counter() - t0) / k * 1e6)
                    if g is not keep:
                        del g
            for m, v in res.items():
                print(json.dumps({"envs": n, "k": k, "method": m, "us_per_step_median": round(statistics.median(v), 3),
                                  "us_per_step_min": round(min(v), 3), "reps": len(v)}), flush=True)


if __name__ == "__main__":
    main()
