#!/usr/bin/env python
"""The product's multi-process path, end to end (BASELINE config 4's layout,
reference "parallel games": delivery_drone/socket_server.py:113-124).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 tools/multirank_check.py --backend gloo --out gpurun_out/mr

Every rank runs VecDroneEnv(count, env_id_base=start) on its shard of
`--total` drones (sharding.shard_bounds) for `--frames` frames: the first half
as one dd_rollout launch with in-kernel Philox actions, the second half as
dd_step launches with actions drawn for the whole batch (a seeded generator)
and sliced to the shard.  Then sharding.gather_obs moves every shard's last
observation block to rank 0 (RCCL with --backend nccl: one GPU per rank;
gloo: host tensors, which lets two ranks share one GPU), and the per-rank
state checksums are gathered too.  Rank 0 runs the same frames as ONE batch in
a fresh child process (`--single`) and compares bit for bit: observations,
rewards, done flags and every SoA field.  Rank 0 writes <out>/multirank.json.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "reinforcement-learning-101_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

FIELDS = ("x", "y", "vx", "vy", "angle", "omega", "fuel", "px", "py", "total_reward", "status", "steps", "episode")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--backend", choices=("gloo", "nccl"), default="gloo")
    p.add_argument("--total", type=int, default=2 * 262_144 + 777)  # ragged: shards differ by one
    p.add_argument("--frames", type=int, default=200)
    p.add_argument("--seed", type=int, default=5)
    p.add_argument("--out", default="gpurun_out/multirank")
    p.add_argument("--single", action="store_true", help="(internal) the one-batch run, saved to --out")
    return p.parse_args()


def run(env, start, count, total, frames, seed, dev):
    """The frames every rank (and the single batch) runs; returns the last
    frame's (obs, reward, done) of this batch."""
    import torch
    half = frames // 2
    obs, reward, done = env.rollout(frames=half, action_seed=seed)
    out = (obs[-1], reward[-1], done[-1]) if half else None
    g = torch.Generator(device=dev).manual_seed(seed)
    for _ in range(frames - half):
        a = torch.randint(0, 8, (total,), device=dev, generator=g, dtype=torch.uint8)  # whole-batch actions
        o, r, d, _ = env.step(a[start:start + count])
        out = (o, r, d)
    return out


def make_env(count, start, seed, dev):
    from delivery_drone_amd import EnvConfig, VecDroneEnv
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=seed)
    env = VecDroneEnv(count, device=dev, config=cfg, env_id_base=start)
    env.reset()
    return env


def single(args):
    import numpy as np
    import torch
    dev = torch.device("cuda", 0)
    env = make_env(args.total, 0, args.seed, dev)
    o, r, d = run(env, 0, args.total, args.total, args.frames, args.seed, dev)
    torch.cuda.synchronize(dev)
    np.savez(os.path.join(args.out, "single.npz"), obs=o.cpu().numpy(), reward=r.cpu().numpy(),
             done=d.cpu().numpy(), **{f: getattr(env, f).cpu().numpy() for f in FIELDS})


def main():
    args = parse()
    os.makedirs(args.out, exist_ok=True)
    if args.single:
        return single(args)
    import numpy as np
    import torch
    import torch.distributed as dist
    from delivery_drone_amd.sharding import dist_env, gather_obs, gather_state, shard_bounds

    rank, world, local = dist_env()
    ndev = torch.cuda.device_count()
    if args.backend == "nccl" and world > ndev:
        raise SystemExit(f"nccl: {world} ranks need {world} GPUs, {ndev} visible")
    dev = torch.device("cuda", local % ndev)
    torch.cuda.set_device(dev)
    if args.backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    start, count = shard_bounds(args.total, rank, world)
    env = make_env(count, start, args.seed, dev)
    t0 = time.perf_counter()
    o, r, d = run(env, start, count, args.total, args.frames, args.seed, dev)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    host = args.backend == "gloo"

    t1 = time.perf_counter()
    g_obs = gather_obs(o.cpu() if host else o, args.total, dst=0)
    gather_s = time.perf_counter() - t1
    payload = {"reward": r.to(torch.float32), "done": d.to(torch.int32)}
    payload.update({f: getattr(env, f).to(torch.float64 if f in FIELDS[:10] else torch.int32) for f in FIELDS})
    g_all = gather_state({k: (v.cpu() if host else v) for k, v in payload.items()}, args.total, dst=0)
    if rank == 0:
        g_rew, g_done = g_all["reward"], g_all["done"]
        g_state = {f: g_all[f] for f in FIELDS}
    if rank == 0:
        child = subprocess.run([sys.executable, os.path.abspath(__file__), "--single", "--total", str(args.total),
                                "--frames", str(args.frames), "--seed", str(args.seed), "--out", args.out],
                               capture_output=True, text=True, timeout=600)
        if child.returncode != 0:
            raise SystemExit(f"single-batch child failed: {child.stderr[-2000:]}")
        ref = np.load(os.path.join(args.out, "single.npz"))
        checks = {
            "obs": bool(np.array_equal(g_obs.cpu().numpy(), ref["obs"])),
            "reward": bool(np.array_equal(g_rew.cpu().numpy().reshape(-1), ref["reward"].astype(np.float32))),
            "done": bool(np.array_equal(g_done.cpu().numpy().reshape(-1), ref["done"].astype(np.int32))),
        }
        for f in FIELDS:
            want = ref[f].astype(np.float64 if f in FIELDS[:10] else np.int32)
            checks[f] = bool(np.array_equal(g_state[f].cpu().numpy().reshape(-1), want))
        res = {"world": world, "backend": args.backend, "devices": [str(dev)] if world == 1 else
               f"{min(world, ndev)} GPU(s) for {world} ranks", "total": args.total, "frames": args.frames,
               "shards": [shard_bounds(args.total, q, world) for q in range(world)],
               "episodes_max": int(ref["episode"].max()), "rank0_frames_s": round(dt, 3),
               "gather_obs_ms": round(gather_s * 1e3, 3), "checks": checks, "bit_equal": all(checks.values()),
               "single_batch": "fresh child process, one VecDroneEnv of all drones"}
        with open(os.path.join(args.out, "multirank.json"), "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res), flush=True)
        ok = res["bit_equal"]
    else:
        ok = True
    dist.barrier()
    dist.destroy_process_group()
    if not ok:
        raise SystemExit("multi-rank result differs from the single batch")


if __name__ == "__main__":
    main()
