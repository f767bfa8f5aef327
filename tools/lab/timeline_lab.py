#!/usr/bin/env python
"""Per-wave timeline of one dd_step launch (lab builds with -DDD_EXP_TIMELINE).

Each wave records the 100 MHz real-time clock at entry (t0), when its loads
have landed (t1), when the frame is done (t2), when its obs rows are issued
(t3) and when its stores are acknowledged (t4), plus HW_ID / XCC_ID.  This
prints, per variant and batch size, the phase percentiles relative to the
first wave's entry and how the co-resident waves of one SIMD overlap.

    python tools/lab/timeline_lab.py --variants tl,tlnomath --envs 262144
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "reinforcement-learning-101_amd"))

import torch  # noqa: E402

from delivery_drone_amd import EnvConfig, VecDroneEnv, abi  # noqa: E402

LAB = os.path.join(REPO, "reinforcement-learning-101_amd", "delivery_drone_amd", "_native", "lab")
TICK_US = 0.01  # s_memrealtime runs at 100 MHz


def pct(a, qs=(0, 10, 50, 90, 100)):
    return [round(float(np.percentile(a, q)), 3) for q in qs]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variants", default="tl")
    p.add_argument("--envs", default="262144")
    p.add_argument("--graph-steps", type=int, default=20)
    p.add_argument("--rounds", type=int, default=8)
    p.add_argument("--out", default="")
    args = p.parse_args()
    dev = torch.device("cuda", 0)
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=0)
    raw = {}
    for n in [int(x) for x in args.envs.split(",")]:
        waves = (n + 63) // 64
        rows = torch.randint(0, 8, (8, n), device=dev, dtype=torch.uint8)
        stream = torch.cuda.Stream(dev)
        runs = {}
        for name in args.variants.split(","):
            lib = abi.load(os.path.join(LAB, f"lib_{name}.so"))
            lib.dd_lab_timeline.argtypes = [ctypes.c_void_p, ctypes.c_int64]
            env = VecDroneEnv(n, device=dev, config=cfg, library=lib)
            env.reset()
            with torch.cuda.stream(stream):
                for k in range(3):
                    env.step(rows[k])
                torch.cuda.synchronize(dev)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=stream):
                    for k in range(args.graph_steps):
                        env.step(rows[k % 8])
                g.replay()
            torch.cuda.synchronize(dev)
            runs[name] = (lib, env, g, [], [])
        names = list(runs)
        for rnd in range(args.rounds):  # ABBA order
            for name in (names if rnd % 2 == 0 else names[::-1]):
                lib, env, g, times, tls = runs[name]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                with torch.cuda.stream(stream):
                    e0.record(stream)
                    g.replay()
                    e1.record(stream)
                torch.cuda.synchronize(dev)
                times.append(e0.elapsed_time(e1) * 1e3 / args.graph_steps)
                buf = np.zeros((min(waves, 1 << 14), 8), dtype=np.uint64)
                rc = lib.dd_lab_timeline(buf.ctypes.data, buf.nbytes)
                if rc != 0:
                    raise SystemExit(f"dd_lab_timeline: {rc}")
                tls.append(buf)
        for name, (lib, env, g, times, tls) in runs.items():
            raw[f"{name}_{n}"] = np.stack(tls)
            spans = []
            for buf in tls:
                spans.append(float((int(buf[:, 4].max()) - int(buf[:, 0].min())) * TICK_US))
            buf = tls[len(tls) // 2]
            t = (buf[:, :5].astype(np.int64) - int(buf[:, 0].min())) * TICK_US
            hw = buf[:, 7].astype(np.uint64)
            hwid = (hw & np.uint64(0xFFFFFFFF)).astype(np.int64)
            xcc = (hw >> np.uint64(32)).astype(np.int64) & 0xF
            simd_key = xcc * 4096 + ((hwid >> 8) & 0xFF) * 4 + ((hwid >> 4) & 3)
            order = np.argsort(simd_key, kind="stable")
            keys, starts, counts = np.unique(simd_key[order], return_index=True, return_counts=True)
            spread_t2 = [t[order[s:s + c], 2].max() - t[order[s:s + c], 2].min() for s, c in zip(starts, counts)]
            med = float(np.median(times))
            res = {
                "variant": name, "envs": n, "us_per_step_median": round(med, 3),
                "us_per_step_min": round(min(times), 3),
                "span_us_median": round(float(np.median(spans)), 3),
                "outside_span_us": round(med - float(np.median(spans)), 3),
                "t1_loaded_pct": pct(t[:, 1]), "t2_frame_done_pct": pct(t[:, 2]),
                "t4_stores_acked_pct": pct(t[:, 4]),
                "load_wait_us_pct": pct(t[:, 1] - t[:, 0]), "frame_us_pct": pct(t[:, 2] - t[:, 1]),
                "store_drain_us_pct": pct(t[:, 4] - t[:, 2]),
                "waves_per_simd": pct(counts), "simd_t2_spread_us_pct": pct(np.array(spread_t2)),
            }
            print(json.dumps(res), flush=True)
        del runs
        torch.cuda.empty_cache()
    if args.out:
        np.savez_compressed(args.out, **raw)


if __name__ == "__main__":
    main()
