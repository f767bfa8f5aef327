#!/usr/bin/env python
"""Lab: is the 16.8M step's allocation spread (DESIGN.md
§4.1 "Placement") steadier when the SoA lives in physically contiguous
memory?  Variants, each its own env at N drones, every field carved from one
slab (field k at a 2 MiB boundary, tools/lab/diag_alloc.rebind_slab's layout):

  torch   the slab from torch's caching allocator (hipMalloc underneath)
  contig  the slab from hipExtMallocWithFlags(hipDeviceMallocContiguous),
          wrapped for torch through __cuda_array_interface__
  V:S     variant V with field k at a 2 MiB boundary + k * S bytes

`--allocs A` envs of each variant, allocated alternately; all are timed in
interleaved rounds (order reversed every other round), graphs of G steps.
One JSON line per env: median / min us per step, allocation order.

    python tools/lab/contig_lab.py --envs 16777216 --allocs 3
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "reinforcement-learning-101_amd"), os.path.dirname(os.path.abspath(__file__))]
import torch  # noqa: E402

from delivery_drone_amd import EnvConfig, VecDroneEnv, abi  # noqa: E402
from delivery_drone_amd.vec_env import _FLOAT_FIELDS  # noqa: E402

HIP_DEVICE_MALLOC_CONTIGUOUS = 0x4


class _DevBuf:
    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False), "version": 3}


def hip_runtime():
    with open("/proc/self/maps") as f:
        for line in f:
            if "libamdhip64.so" in line:
                return ctypes.CDLL(line.split()[-1])
    raise RuntimeError("libamdhip64.so is not mapped")


def rebind(env, how, hip, keep):
    """how: "torch" / "contig", optionally ":S" — field k then starts at a
    2 MiB boundary + k * S bytes (in a contiguous range: a physical stagger)."""
    how, _, stagger = how.partition(":")
    stagger = int(stagger or 0)
    names = list(_FLOAT_FIELDS) + ["status", "steps", "episode", "obs", "reward", "_done"]
    tens = [getattr(env, k) for k in names]
    align = 2 << 20
    offs, pos = [], 0
    for k, t in enumerate(tens):
        pos = (pos + align - 1) // align * align + k * stagger
        offs.append(pos)
        pos += t.numel() * t.element_size()
    total = pos + align
    if how == "contig":
        p = ctypes.c_void_p()
        rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(total), ctypes.c_uint(HIP_DEVICE_MALLOC_CONTIGUOUS))
        if rc != 0:
            raise RuntimeError(f"hipExtMallocWithFlags(contiguous, {total} B): hipError {rc}")
        slab = torch.as_tensor(_DevBuf(p.value, total), device=env.device)
        keep.append(p)
    else:
        slab = torch.empty(total, dtype=torch.uint8, device=env.device)
    for name, t, o in zip(names, tens, offs):
        nb = t.numel() * t.element_size()
        v = slab[o:o + nb].view(t.dtype).view(t.shape)
        v.copy_(t)
        setattr(env, name, v)
    env._slab = slab
    env._state = abi.DDState(
        *[ctypes.c_void_p(getattr(env, f).data_ptr()) for f in _FLOAT_FIELDS],
        ctypes.c_void_p(env.status.data_ptr()), ctypes.c_void_p(env.steps.data_ptr()),
        ctypes.c_void_p(env.episode.data_ptr()), env.env_id_base, abi.DD_F32, 0)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=16_777_216)
    p.add_argument("--allocs", type=int, default=3)
    p.add_argument("--variants", default="torch,contig")
    p.add_argument("--graph-steps", type=int, default=10)
    p.add_argument("--rounds", type=int, default=12)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    n = a.envs
    hip = hip_runtime()
    keep = []
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=0)
    rows = torch.randint(0, 8, (4, n), device=dev, dtype=torch.uint8)
    stream = torch.cuda.Stream(dev)
    runs = []
    for k in range(a.allocs):
        for v in a.variants.split(","):
            env = VecDroneEnv(n, device=dev, config=cfg)
            env.reset()
            rebind(env, v, hip, keep)
            torch.cuda.empty_cache()
            with torch.cuda.stream(stream):
                for j in range(3):
                    env.step(rows[j % 4])
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=stream):
                    for j in range(a.graph_steps):
                        env.step(rows[j % 4])
            runs.append((f"{v}{k}", env, g, []))
    torch.cuda.synchronize()
    for rnd in range(a.rounds):
        for name, env, g, ts in (runs if rnd % 2 == 0 else runs[::-1]):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(stream):
                e0.record(stream)
                g.replay()
                e1.record(stream)
            torch.cuda.synchronize()
            if rnd >= 2:
                ts.append(e0.elapsed_time(e1) * 1e3 / a.graph_steps)
    bpe = 147
    for i, (name, env, g, ts) in enumerate(runs):
        us = statistics.median(ts)
        print(json.dumps({"envs": n, "env": name, "alloc_order": i, "us_median": round(us, 2),
                          "us_min": round(min(ts), 2), "frac": round(bpe * n / (us * 1e-6) / 8e12, 4),
                          "slab_ptr": hex(env._slab.data_ptr())}), flush=True)
    torch.cuda.synchronize()  # the contiguous slabs go with the process


if __name__ == "__main__":
    main()
