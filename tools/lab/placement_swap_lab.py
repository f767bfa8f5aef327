#!/usr/bin/env python
"""Diagnostic: at 16.8M drones, is the placement-dependent step time a
property of the state arrays or of the output arrays (obs rows, reward,
done)?  Three envs are allocated; each (state of env i, outputs of env j)
pair is stepped through VecDroneEnv.step(out=...) and timed in interleaved
rounds (hipGraph replays, HIP events)."""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "reinforcement-learning-101_amd"))
import torch  # noqa: E402
from delivery_drone_amd import EnvConfig, VecDroneEnv  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16_777_216
    dev = torch.device("cuda", 0)
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=0)
    rows = torch.randint(0, 8, (4, n), device=dev, dtype=torch.uint8)
    envs = []
    for _ in range(3):
        e = VecDroneEnv(n, device=dev, config=cfg)
        e.reset()
        envs.append(e)
    stream = torch.cuda.Stream(dev)
    pairs = [(i, j) for i in range(3) for j in range(3)]
    graphs = {}
    for i, j in pairs:
        st, ou = envs[i], envs[j]
        out = (ou.obs, ou.reward, ou.done)
        with torch.cuda.stream(stream):
            for k in range(2):
                st.step(rows[k % 4], out=out)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                for k in range(10):
                    st.step(rows[k % 4], out=out)
        graphs[(i, j)] = (g, [])
    torch.cuda.synchronize()
    for rnd in range(8):
        order = pairs if rnd % 2 == 0 else pairs[::-1]
        for p in order:
            g, ts = graphs[p]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(stream):
                e0.record(stream)
                g.replay()
                g.replay()
                e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / 20)
    for (i, j), (g, ts) in graphs.items():
        print(json.dumps({"state_of_env": i, "outputs_of_env": j, "us_median": round(statistics.median(ts), 1),
                          "us_min": round(min(ts), 1)}), flush=True)


if __name__ == "__main__":
    main()
