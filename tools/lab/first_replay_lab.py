#!/usr/bin/env python
"""Is a hipGraph's FIRST replay slower than later ones?  The driver's K = 20
bench line times the 20-step graph's first replay (bench.py warms up with a
5-step graph).  Per trial: a fresh VecDroneEnv at config 3, the 5-step and
the 20-step graphs captured as bench.py captures them, the 5-step graph
replayed (the warmup), then the 20-step graph replayed three times, each
timed by the wall clock (replay + synchronize) and by events on the stream.

  mode plain   as bench.py
  mode upload  hipGraphUpload of the 20-step exec handle after capture
  mode touch   the 20-step graph's kernel-argument pages warmed by replaying
               a graph captured from the same env with the same arguments
               (a learning aid only: it runs extra steps)"""
import ctypes
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "reinforcement-learning-101_amd"))
import torch  # noqa: E402
from delivery_drone_amd import EnvConfig, VecDroneEnv  # noqa: E402

_hip = ctypes.CDLL("libamdhip64.so")
_hip.hipGraphUpload.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
_hip.hipGraphUpload.restype = ctypes.c_int


def trial(mode, n=262144, k=20, w=5):
    dev = torch.device("cuda", 0)
    env = VecDroneEnv(n, device=dev, config=EnvConfig(randomize_drone=True, randomize_platform=True,
                                                      auto_reset=True, seed=0))
    env.reset()
    rows = torch.randint(0, 8, (64, n), device=dev, dtype=torch.uint8)
    stream = torch.cuda.Stream(dev)
    stream.wait_stream(torch.cuda.current_stream(dev))
    graphs = {}
    with torch.cuda.stream(stream):
        for i in range(3):
            env.step(rows[i])
        torch.cuda.synchronize(dev)
        for m in (k, w) + ((k + 1,) if mode == "touch" else ()):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                for i in range(m):
                    env.step(rows[i % 64])
            graphs[m] = g
        if mode == "upload":
            rc = _hip.hipGraphUpload(ctypes.c_void_p(graphs[k].raw_cuda_graph_exec()),
                                     ctypes.c_void_p(stream.cuda_stream))
            assert rc == 0, rc
        if mode == "touch":
            graphs[k + 1].replay()
        graphs[w].replay()  # the warmup
        torch.cuda.synchronize(dev)
        wall, dev_us = [], []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            e0.record(stream)
            graphs[k].replay()
            e1.record(stream)
            torch.cuda.synchronize(dev)
            wall.append((time.perf_counter() - t0) * 1e6)
            dev_us.append(e0.elapsed_time(e1) * 1e3)
    del graphs, env
    torch.cuda.empty_cache()
    return wall, dev_us


def main():
    modes = ["plain", "upload", "touch"]
    res = {m: [] for m in modes}
    for t in range(8):
        for m in (modes if t % 2 == 0 else modes[::-1]):
            res[m].append(trial(m))
    for m, rows in res.items():
        out = {"mode": m, "trials": len(rows)}
        for j in range(3):
            out[f"wall_{j}"] = round(statistics.median(r[0][j] for r in rows), 1)
            out[f"events_{j}"] = round(statistics.median(r[1][j] for r in rows), 1)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
