#!/usr/bin/env python
"""Wall clock of K config-3 steps by launch method, the bench's timed-region
shape (device sync, K steps, device sync; perf_counter around it):

  graph_ev     hipGraphs of min(50, K) dd_step with head / tail event-record
               nodes added after capture (span_events.KernelSpanEvents: the
               bench's kernel-span timing until the stamps replaced it)
  graph_stamp  the same graphs with dd_stamp kernels captured at the head and
               tail (bench.KernelSpanStamps: the bench's timing now)
  graph        the same graphs with no markers
  direct       K dd_step calls straight through ctypes (prebuilt argument
               structs, one per action row), no graph
  ramp:A+B+..  plain graphs of A, then B, ... steps (the last size repeated
               until K): a small first graph starts the GPU sooner

Prints one JSON line per (K, method): median / min wall us per step over R
repetitions, the host submission time per step (perf_counter after the last
launch call, before the sync) and, for the marked methods, the kernels' own
us per launch from the markers (span minus the span of a graph of the two
markers alone).

    python tools/lab/launch_probe.py --ks 20,200,2000 --reps 15
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time
import warnings

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "reinforcement-learning-101_amd"), os.path.dirname(os.path.abspath(__file__))]

import torch  # noqa: E402
from span_events import KernelSpanEvents  # noqa: E402

import bench  # noqa: E402
from delivery_drone_amd import EnvConfig, VecDroneEnv, abi  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=262144)
    p.add_argument("--ks", default="20,200,2000")
    p.add_argument("--reps", type=int, default=15)
    p.add_argument("--rows", type=int, default=8)
    p.add_argument("--methods", default="graph_ev,graph_stamp,graph,direct")
    p.add_argument("--sched", default="", choices=["", "auto", "spin", "yield"],
                   help="hipSetDeviceFlags(hipDeviceSchedule*) before the first GPU work (default: leave it)")
    args = p.parse_args()
    dev = torch.device("cuda", 0)
    if args.sched:
        torch.cuda.init()
        events0 = KernelSpanEvents()  # the HIP runtime torch loaded
        flag = {"auto": 0, "spin": 1, "yield": 2}[args.sched]
        rc = events0.hip.hipSetDeviceFlags(ctypes.c_uint(flag))
        print(json.dumps({"sched": args.sched, "hipSetDeviceFlags_rc": rc}), flush=True)
        events0.close()
    n = args.envs
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=0)
    env = VecDroneEnv(n, device=dev, config=cfg)
    env.reset()
    rows = torch.randint(0, 8, (args.rows, n), device=dev, dtype=torch.uint8)
    stream = torch.cuda.Stream(dev)
    stream.wait_stream(torch.cuda.current_stream(dev))
    events = KernelSpanEvents()
    stamps = bench.KernelSpanStamps(env._lib, dev)
    lib = env._lib
    with torch.cuda.stream(stream):
        for _ in range(3):
            env.step(rows[0])
        torch.cuda.synchronize(dev)
        ios = []  # prebuilt dd_step arguments, one io struct per action row
        for r in range(args.rows):
            env.step(rows[r])
            ios.append(abi.DDStepIO.from_buffer_copy(env._io))
        cfg_ref, st_ref = ctypes.byref(env._cfg), ctypes.byref(env._state)
        io_refs = [ctypes.byref(io) for io in ios]
        sh = ctypes.c_void_p(stream.cuda_stream)
        fn = lib.dd_step
        graphs = {}

        def graph(k, mark, head, tail):
            key = (k, mark, head, tail)
            if key not in graphs:
                ev = mark == "ev" and (head or tail)
                g = torch.cuda.CUDAGraph(keep_graph=ev)
                with warnings.catch_warnings():
                    warnings.simplefilter("ignore")  # an empty capture (the event calibration graph)
                    with torch.cuda.graph(g, stream=stream):
                        if mark == "stamp" and head:
                            stamps.stamp(0, stream)
                        for i in range(k):
                            env.step(rows[i % args.rows])
                        if mark == "stamp" and tail:
                            stamps.stamp(1, stream)
                if ev:
                    events.add_nodes(g, head, tail)
                    g.instantiate()
                graphs[key] = g
            return graphs[key]

        def run(method, k):
            if method.startswith("ramp:"):  # graphs of the given sizes in turn (the last one repeated to K)
                sizes = [int(x) for x in method[5:].split("+")]
                seq, left = [], k
                while left > 0:
                    x = min(sizes[min(len(seq), len(sizes) - 1)], left)
                    seq.append(x)
                    left -= x
                for g in [graph(x, None, False, False) for x in seq]:
                    g.replay()
                return
            if method.startswith("graph"):
                mark = {"graph_ev": "ev", "graph_stamp": "stamp"}.get(method)
                G = min(50, k)
                seq = [G] * (k // G) + ([k % G] if k % G else [])
                gs = [graph(x, mark, mark is not None and j == 0, mark is not None and j == len(seq) - 1)
                      for j, x in enumerate(seq)]
                for g in gs:
                    g.replay()
            else:
                for i in range(k):
                    rc = fn(cfg_ref, st_ref, io_refs[i % args.rows], n, sh)
                    if rc:
                        raise RuntimeError(f"dd_step rc {rc}")

        def span_ms(method):
            return events.elapsed_ms() if method == "graph_ev" else stamps.elapsed_ms(0, 1)

        # the markers alone: a graph of the two event nodes / the two stamps
        cal = {}
        ge = graph(0, "ev", True, True)
        gs = graph(0, "stamp", True, True)
        for method, g in (("graph_ev", ge), ("graph_stamp", gs)):
            v = []
            for _ in range(9):
                g.replay()
                v.append(span_ms(method))
            cal[method] = statistics.median(v)

        methods = args.methods.split(",")
        for k in [int(x) for x in args.ks.split(",")]:
            for m in methods:  # build + warm
                run(m, k)
            torch.cuda.synchronize(dev)
            res = {m: ([], [], []) for m in methods}
            for rep in range(args.reps):
                for m in (methods if rep % 2 == 0 else methods[::-1]):
                    run("graph", 5)  # the warm-up, as bench.py's
                    torch.cuda.synchronize(dev)
                    t0 = time.perf_counter()
                    run(m, k)
                    t1 = time.perf_counter()
                    torch.cuda.synchronize(dev)
                    t2 = time.perf_counter()
                    res[m][0].append((t2 - t0) / k * 1e6)
                    res[m][1].append((t1 - t0) / k * 1e6)
                    if m in cal:
                        res[m][2].append((span_ms(m) - cal[m]) / k * 1e3)
            for m in methods:
                w, h, kern = res[m]
                row = {"envs": n, "k": k, "method": m, "sched": args.sched or "default", "us_per_step_median": round(statistics.median(w), 3),
                       "us_per_step_min": round(min(w), 3),
                       "steps_per_s_median": round(n / (statistics.median(w) * 1e-6), 1),
                       "host_submit_us_per_step": round(statistics.median(h), 3)}
                if kern:
                    row["kernel_us_per_launch_median"] = round(statistics.median(kern), 3)
                    row["marker_cal_us"] = round(cal[m] * 1e3, 2)
                print(json.dumps(row), flush=True)
    events.close()


if __name__ == "__main__":
    main()
