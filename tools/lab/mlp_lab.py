#!/usr/bin/env python
"""A/B timing of dd_mlp_forward builds (actor + sampling), interleaved rounds."""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "reinforcement-learning-101_amd"))
import torch  # noqa: E402
from torch import nn  # noqa: E402
from delivery_drone_amd import MlpNet, abi  # noqa: E402

LAB = os.path.join(REPO, "reinforcement-learning-101_amd", "delivery_drone_amd", "_native", "lab")
FLOPS = 2 * (15 * 128 + 128 * 128 + 128 * 64 + 64 * 3)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variants", default="base")
    p.add_argument("--rows", default="65536,262144")
    p.add_argument("--rounds", type=int, default=15)
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--compute", default="f32", help="f32 or f16x3 (variants built before ABI 6 take f32 only)")
    args = p.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = nn.Sequential(nn.Linear(15, 128), nn.LayerNorm(128), nn.ReLU(), nn.Linear(128, 128), nn.LayerNorm(128),
                        nn.ReLU(), nn.Linear(128, 64), nn.LayerNorm(64), nn.ReLU(), nn.Linear(64, 3))
    sd = net.state_dict()
    for n in [int(x) for x in args.rows.split(",")]:
        obs = torch.randn(n, 15, device=dev)
        acts = torch.empty(n, dtype=torch.uint8, device=dev)
        lp = torch.empty(n, device=dev)
        nets = {v: (MlpNet(sd, device=dev, compute=args.compute,
                           library=abi.load(os.path.join(LAB, f"lib_{v}.so"))), [])
                for v in args.variants.split(",")}
        ref = None
        for v, (m, _) in nets.items():
            m.act(obs, actions_out=acts, log_prob_out=lp)
            pr = m(obs)
            if ref is None:
                ref = pr.clone()
            err = (pr - ref).abs().max().item()
            if err > 1e-5:
                print(json.dumps({"variant": v, "rows": n, "MISMATCH": err}), flush=True)
        torch.cuda.synchronize()
        # each variant's `reps` calls captured in a hipGraph: device time, not the
        # host's launch rate (eager calls cost ~9 us each on the host)
        stream = torch.cuda.Stream(dev)
        graphs = {}
        for v, (m, _) in nets.items():
            with torch.cuda.stream(stream):
                m.act(obs, actions_out=acts, log_prob_out=lp)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=stream):
                    for s in range(args.reps):
                        m.act(obs, step=s, actions_out=acts, log_prob_out=lp)
                g.replay()
            graphs[v] = g
        torch.cuda.synchronize()
        names = list(nets)
        for rnd in range(args.rounds):  # ABBA: alternate the order so position effects cancel
            for v in (names if rnd % 2 == 0 else names[::-1]):
                m, ts = nets[v]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                with torch.cuda.stream(stream):
                    e0.record(stream)
                    graphs[v].replay()
                    e1.record(stream)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / args.reps)
        for v, (m, ts) in nets.items():
            us = statistics.median(ts)
            print(json.dumps({"rows": n, "variant": v, "compute": args.compute, "us_median": round(us, 2), "us_min": round(min(ts), 2),
                              "tflops": round(n * FLOPS / (us * 1e-6) / 1e12, 2)}), flush=True)


if __name__ == "__main__":
    main()
