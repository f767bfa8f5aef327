#!/usr/bin/env python
"""CPU estimate of how often each rare branch of the config-3 step kernel runs
per WAVE (64 consecutive lanes), from the oracle stepping the bench's
workload (random spawn, auto-reset, uniform random 3-bit actions).  A wave
executes a divergent branch when any of its lanes takes it, so the per-wave
rate, not the per-lane one, is what the branch costs in VALU issue.

    python tools/lab/branch_freq.py [--envs 262144 --steps 300 --warm 200]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "reinforcement-learning-101_amd")]
from delivery_drone_amd.config import EnvConfig  # noqa: E402
from oracle.oracle import OracleEnv  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=262_144)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warm", type=int, default=300)
    a = p.parse_args()
    n = a.envs
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=0)
    env = OracleEnv(n, precision="f32", config=cfg)
    env.reset()
    rng = np.random.default_rng(0)
    keys = ["respawn", "main_on", "upright", "near_pad", "wrap", "terminal"]
    lane = {k: 0.0 for k in keys}
    wave = {k: 0.0 for k in keys}
    for t in range(a.warm + a.steps):
        acts = rng.integers(0, 8, n, dtype=np.uint8)
        if t >= a.warm:
            done0 = (env.status & 1) != 0
            live = ~done0
            main = live & ((acts & 1) != 0) & (env.fuel > 0)
            ang = env.angle.astype(np.float64) + env.omega.astype(np.float64)  # before the wrap
            wrap = live & (np.abs(ang) > 180)
        env.step(acts)
        if t >= a.warm:
            upright = live & (np.abs(env.angle) <= 20)
            near = upright & (np.abs(env.x - env.px) <= 61) & (np.abs(env.y - env.py) <= 21)
            term = live & ((env.status & 1) != 0)
            for k, m in zip(keys, (done0, main, upright, near, wrap, term)):
                lane[k] += m.mean() / a.steps
                wave[k] += m[: n // 64 * 64].reshape(-1, 64).any(1).mean() / a.steps
    print(json.dumps({"envs": n, "steps": a.steps, "warm": a.warm,
                      "per_lane": {k: round(v, 5) for k, v in lane.items()},
                      "per_wave": {k: round(v, 4) for k, v in wave.items()}}))


if __name__ == "__main__":
    main()
