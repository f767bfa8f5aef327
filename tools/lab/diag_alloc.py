#!/usr/bin/env python
"""Diagnostic: does the step at 16.8M drones depend on allocation order?
Times three envs allocated one after another, in ABBA-interleaved rounds."""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "reinforcement-learning-101_amd"))
import torch  # noqa: E402
import ctypes  # noqa: E402
from delivery_drone_amd import EnvConfig, VecDroneEnv, abi  # noqa: E402
from delivery_drone_amd.vec_env import _FLOAT_FIELDS  # noqa: E402


def rebind_slab(env, stagger):
    """Move the env's SoA fields and outputs into one allocation, field k
    starting at a 2 MiB boundary + k * stagger bytes."""
    names = list(_FLOAT_FIELDS) + ["status", "steps", "episode", "obs", "reward", "_done"]
    tens = [getattr(env, k) for k in names]
    align = 2 << 20
    offs, pos = [], 0
    for k, t in enumerate(tens):
        nb = t.numel() * t.element_size()
        pos = (pos + align - 1) // align * align + k * stagger
        offs.append(pos)
        pos += nb
    slab = torch.empty(pos + align, dtype=torch.uint8, device=env.device)
    for k, (name, t) in enumerate(zip(names, tens)):
        nb = t.numel() * t.element_size()
        v = slab[offs[k]:offs[k] + nb].view(t.dtype).view(t.shape)
        v.copy_(t)
        setattr(env, name, v)
    env._slab = slab
    env._state = abi.DDState(
        *[ctypes.c_void_p(getattr(env, f).data_ptr()) for f in _FLOAT_FIELDS],
        ctypes.c_void_p(env.status.data_ptr()), ctypes.c_void_p(env.steps.data_ptr()),
        ctypes.c_void_p(env.episode.data_ptr()), env.env_id_base, abi.DD_F32, 0)


def main():
    dev = torch.device("cuda", 0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16_777_216
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=0)
    mode = sys.argv[2] if len(sys.argv) > 2 else "plain"
    pad = None
    if mode in ("pad", "padfree"):  # a large allocation before the envs
        pad = torch.empty(4 << 30, dtype=torch.uint8, device=dev)
        pad.fill_(1)
        if mode == "padfree":
            del pad
            pad = None
            torch.cuda.empty_cache()
    rows = torch.randint(0, 8, (4, n), device=dev, dtype=torch.uint8)
    stream = torch.cuda.Stream(dev)
    runs = []
    envs = []
    for k in range(3):
        env = VecDroneEnv(n, device=dev, config=cfg)
        env.reset()
        if mode.startswith("slab"):
            rebind_slab(env, int(mode[4:] or 0))
            torch.cuda.empty_cache()
        envs.append(env)
    order = [2, 1, 0] if mode == "revgraph" else [0, 1, 2]
    runs = [None] * 3
    for k in order:
        env = envs[k]
        with torch.cuda.stream(stream):
            for j in range(3):
                env.step(rows[j % 4])
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                for j in range(10):
                    env.step(rows[j % 4])
        runs[k] = (env, g, [])
    torch.cuda.synchronize()
    for rnd in range(10):
        order = range(3) if rnd % 2 == 0 else reversed(range(3))
        for k in order:
            env, g, ts = runs[k]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(stream):
                e0.record(stream)
                g.replay()
                e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / 10)
    for k, (env, g, ts) in enumerate(runs):
        print(json.dumps({"mode": mode, "env": k, "obs_ptr": hex(env.obs.data_ptr()), "x_ptr": hex(env.x.data_ptr()),
                          "us_median": round(statistics.median(ts), 2), "us_min": round(min(ts), 2)}), flush=True)


if __name__ == "__main__":
    main()
