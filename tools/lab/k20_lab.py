#!/usr/bin/env python
"""Host-side overheads of a short timed region (the driver's `--steps 20 --warmup 5`).

For config 3 (262,144 drones) this times K = 20 steps replayed from one
captured hipGraph, the way bench.py does, under a few variants of what
happens before the timed replay:

  first      the graph's first replay is the timed one (bench.py at K=20)
  uploaded   hipGraphUpload on the graph before the warmup (no launch)
  second     the graph replayed once untimed before the warmup

Each prints wall (host perf_counter around replay + synchronize) and device
(HIP events on the replay stream) microseconds per step.  DD_SYNC=spin|yield|
blocking sets hipSetDeviceFlags before the device is initialised.
"""
import ctypes
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "reinforcement-learning-101_amd"))

_hip = ctypes.CDLL("libamdhip64.so")
_FLAGS = {"spin": 1, "yield": 2, "blocking": 4}
mode = os.environ.get("DD_SYNC", "")
if mode:
    rc = _hip.hipSetDeviceFlags(ctypes.c_uint(_FLAGS[mode]))
    print(f"hipSetDeviceFlags({mode}) -> {rc}", file=sys.stderr)

import torch  # noqa: E402

from delivery_drone_amd import EnvConfig, VecDroneEnv  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n, K, W = 262_144, 20, 5
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=0)
    env = VecDroneEnv(n, device=dev, config=cfg)
    env.reset()
    rows = torch.randint(0, 8, (64, n), device=dev, dtype=torch.uint8)
    stream = torch.cuda.Stream(dev)
    stream.wait_stream(torch.cuda.current_stream(dev))

    def capture(k):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for i in range(k):
                env.step(rows[i % 64])
        return g

    with torch.cuda.stream(stream):
        for i in range(3):
            env.step(rows[i])
    torch.cuda.synchronize(dev)
    res = {}
    for trial in range(8):
        for variant in ("first", "uploaded", "second"):
            with torch.cuda.stream(stream):
                gk, gw = capture(K), capture(W)
                if variant == "uploaded":
                    _hip.hipGraphUpload(ctypes.c_void_p(gk.raw_cuda_graph_exec()), ctypes.c_void_p(stream.cuda_stream))
                    _hip.hipGraphUpload(ctypes.c_void_p(gw.raw_cuda_graph_exec()), ctypes.c_void_p(stream.cuda_stream))
                elif variant == "second":
                    gk.replay()
                    gw.replay()
                gw.replay()
                torch.cuda.synchronize(dev)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0 = time.perf_counter()
                e0.record(stream)
                gk.replay()
                e1.record(stream)
                torch.cuda.synchronize(dev)
                wall = time.perf_counter() - t0
            res.setdefault(variant, []).append((wall * 1e6 / K, e0.elapsed_time(e1) * 1e3 / K))
    for v, xs in res.items():
        print(json.dumps({"sync": mode or "default", "variant": v,
                          "wall_us_per_step_median": round(statistics.median(x[0] for x in xs), 3),
                          "dev_us_per_step_median": round(statistics.median(x[1] for x in xs), 3),
                          "wall_all": [round(x[0], 2) for x in xs]}), flush=True)


if __name__ == "__main__":
    main()
