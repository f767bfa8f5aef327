#!/usr/bin/env python
"""Bit-compare dd_rollout between two builds (lab A/B correctness gate).

Both builds start from the same state and actions; obs, reward, done and the
final state must be identical in every bit.  Also dd_step (one launch per
frame, 200 frames after a 300-frame warm-up) at 262,144 and 4,100 lanes, both
storage widths: every frame's obs, reward, done and the final state.  Frame counts cover the prologue
and epilogue cases (1, 2, 3, odd, even), both auto-reset and sticky done,
tensor and in-kernel Philox actions, and a ragged batch.

    python tools/lib_equal_check.py --a base --b obslag
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "reinforcement-learning-101_amd"))
import torch  # noqa: E402
from delivery_drone_amd import EnvConfig, VecDroneEnv, abi  # noqa: E402

LAB = os.path.join(REPO, "reinforcement-learning-101_amd", "delivery_drone_amd", "_native", "lab")


def run(lib, n, frames, auto, philox, start, acts, dev):
    cfg = EnvConfig(randomize_drone=True, auto_reset=auto, seed=3)
    e = VecDroneEnv(n, device=dev, config=cfg)
    e._lib = abi.load(os.path.join(LAB, f"lib_{lib}.so"), abi_versions=(11, 12))
    e.load_state_dict(start)
    obs = torch.full((frames, n, 15), float("nan"), device=dev)
    rew = torch.empty(frames, n, device=dev)
    done = torch.empty(frames, n, device=dev, dtype=torch.bool)
    e.rollout(None if philox else acts[:frames], frames=frames, obs_out=obs, reward_out=rew, done_out=done,
              action_seed=11 if philox else None)
    torch.cuda.synchronize()
    return obs, rew, done, e.state_dict()


def run_steps(lib, n, frames, precision, start, acts, dev):
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=5)
    e = VecDroneEnv(n, device=dev, config=cfg, precision=precision)
    e._lib = abi.load(os.path.join(LAB, f"lib_{lib}.so"), abi_versions=(11, 12))
    e.load_state_dict(start)
    outs = []
    for t in range(frames):
        o, r, d, _ = e.step(acts[t])
        outs.append((o.clone(), r.clone(), d.clone()))
    torch.cuda.synchronize()
    return outs, e.state_dict()


def step_cases(a, b, dev):
    bad = 0
    for n in (262_144, 4_100):
        for precision in ("f32", "f64"):
            cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=5)
            base_env = VecDroneEnv(n, device=dev, config=cfg, precision=precision)
            base_env.reset()
            base_env.rollout(torch.randint(0, 8, (300, n), device=dev, dtype=torch.uint8), frames=300)
            start = base_env.state_dict()
            acts = torch.randint(0, 8, (200, n), device=dev, dtype=torch.uint8)
            oa, sa = run_steps(a, n, 200, precision, start, acts, dev)
            ob, sb = run_steps(b, n, 200, precision, start, acts, dev)
            eq = {"obs": all(torch.equal(x[0].view(torch.int32), y[0].view(torch.int32)) for x, y in zip(oa, ob)),
                  "reward": all(torch.equal(x[1], y[1]) for x, y in zip(oa, ob)),
                  "done": all(torch.equal(x[2], y[2]) for x, y in zip(oa, ob)),
                  "state": all(torch.equal(sa[k], sb[k]) for k in sa)}
            ok = all(eq.values())
            bad += not ok
            print(json.dumps({"kernel": "step", "n": n, "precision": precision, "frames": 200, "ok": ok, **eq}),
                  flush=True)
    return bad


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--a", default="base")
    p.add_argument("--b", default="obslag")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    bad = step_cases(a.a, a.b, dev)
    for n in (65_536, 4_100):
        for auto in (True, False):
            base_env = VecDroneEnv(n, device=dev, config=EnvConfig(randomize_drone=True, auto_reset=auto, seed=3))
            base_env.reset()
            # some frames first so lanes are mid-episode, some done
            base_env.rollout(torch.randint(0, 8, (300, n), device=dev, dtype=torch.uint8), frames=300)
            start = base_env.state_dict()
            acts = torch.randint(0, 8, (256, n), device=dev, dtype=torch.uint8)
            for frames in (1, 2, 3, 4, 7, 64, 255, 256):
                for philox in (False, True):
                    ra = run(a.a, n, frames, auto, philox, start, acts, dev)
                    rb = run(a.b, n, frames, auto, philox, start, acts, dev)
                    eq = {
                        "obs": torch.equal(ra[0].view(torch.int32), rb[0].view(torch.int32)),
                        "reward": torch.equal(ra[1].view(torch.int32), rb[1].view(torch.int32)),
                        "done": torch.equal(ra[2], rb[2]),
                        "state": all(torch.equal(ra[3][k], rb[3][k]) for k in ra[3]),
                        "obs_finite": bool(torch.isfinite(rb[0]).all()),
                    }
                    ok = all(eq.values())
                    bad += not ok
                    print(json.dumps({"n": n, "auto": auto, "frames": frames, "philox": philox, "ok": ok, **eq}),
                          flush=True)
    print(json.dumps({"mismatching_cases": bad}))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
