#!/usr/bin/env python
"""How the event-record nodes bench.py adds to its timed hipGraphs time a
graph: spans of graphs with head/tail event nodes around N config-3 dd_step
kernels, N = 0 (markers only), 1, 2, 5, 10, 20, 40, each replayed R times in
interleaved rounds (first replay reported apart).  A linear fit span = a + N t
gives the markers' fixed cost `a` and the per-kernel time `t`.

    python tools/lab/graph_event_probe.py [--rounds 6]
"""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "reinforcement-learning-101_amd"), os.path.dirname(os.path.abspath(__file__))]
import torch  # noqa: E402
from span_events import KernelSpanEvents  # noqa: E402

from delivery_drone_amd import EnvConfig, VecDroneEnv  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=6)
    p.add_argument("--envs", type=int, default=262_144)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=0)
    env = VecDroneEnv(a.envs, device=dev, config=cfg)
    env.reset()
    rows = torch.randint(0, 8, (8, a.envs), device=dev, dtype=torch.uint8)
    stream = torch.cuda.Stream(dev)
    Ns = [0, 1, 2, 5, 10, 20, 40]
    spans = {n: KernelSpanEvents() for n in Ns}
    graphs = {}
    with torch.cuda.stream(stream):
        for k in range(3):
            env.step(rows[k % 8])
        torch.cuda.synchronize(dev)
        for n in Ns:
            g = torch.cuda.CUDAGraph(keep_graph=True)
            try:
                with torch.cuda.graph(g, stream=stream):
                    for k in range(n):
                        env.step(rows[k % 8])
                spans[n].add_nodes(g, True, True)
                g.instantiate()
            except Exception as e:  # noqa: BLE001  (an empty capture may be refused)
                print(f"N={n}: {type(e).__name__}: {e}", file=sys.stderr)
                continue
            graphs[n] = g
        Ns = [n for n in Ns if n in graphs]
        res = {n: [] for n in Ns}
        for r in range(a.rounds):
            for n in (Ns if r % 2 == 0 else Ns[::-1]):
                graphs[n].replay()
                res[n].append(spans[n].elapsed_ms() * 1e3)
        torch.cuda.synchronize(dev)
    out = {n: {"first_us": round(v[0], 2), "rest_median_us": round(statistics.median(v[1:]), 2)} for n, v in res.items()}
    xs = [n for n in Ns if n > 0]
    ys = [statistics.median(res[n][1:]) for n in xs]
    mx, my = statistics.mean(xs), statistics.mean(ys)
    t = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    print(json.dumps({"spans": out, "fit": {"a_us": round(my - t * mx, 2), "t_us": round(t, 3)}}))


if __name__ == "__main__":
    main()
