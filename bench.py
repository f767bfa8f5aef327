#!/usr/bin/env python
"""Benchmark of the drone step path: env-steps/s per node, HBM roofline, CPU baseline.

    python bench.py [--gpus N --steps K --warmup W]                      # 1 GPU
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N  # N GPUs

A "step" is one frame of every drone on every rank: one ``dd_step`` launch
per GPU over its resident shard (state, actions and outputs already in HBM).
Default workload = BASELINE config 3 per GPU — 262,144 drones, randomised
spawn, auto-reset, uniform random 3-bit actions, the [N,15] observation
written every frame — so N=8 is config 4 (2,097,152 drones, weak scaling).
Steps are replayed from hipGraphs (torch.cuda.CUDAGraph) of min(``--graph-steps``,
K) launches plus one of the remainder; K steps are timed between barriers + device syncs, the max over
ranks is reported.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import multiprocessing as mp
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "reinforcement-learning-101_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "env-steps/sec (whole node), N parallel drones, 1/2/4/8 MI355X; HBM GB/s %peak"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E peak (spec)


def parse():
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--warmup", type=int, default=200)
    p.add_argument("--envs-per-gpu", type=int, default=262_144)
    p.add_argument("--precision", choices=("f32", "f64"), default="f32")
    p.add_argument("--graph-steps", type=int, default=50, help="launches per captured hipGraph (0 = eager)")
    p.add_argument("--no-obs", action="store_true", help="skip the observation write (not the default)")
    p.add_argument("--action-rows", type=int, default=64, help="distinct pre-generated action rows cycled")
    p.add_argument("--cpu-baseline", type=float, default=8.0,
                   help="seconds of CPU-baseline wall time per leg (0 = skip)")
    p.add_argument("--cpu-workers", type=int, default=0,
                   help="CPU-baseline processes per leg (0 = this process's CPU share: host_cpu_share())")
    p.add_argument("--cpu-baseline-json", default="",
                   help="(set by the N > 1 launcher) a cpu_baseline already measured, for rank 0 to report")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                   help="process-group backend for N>1 (nccl = RCCL over xGMI; gloo only to rehearse "
                        "several ranks sharing one GPU)")
    p.add_argument("--rollout-point", type=int, default=65_536,
                   help="also time BASELINE config 5 (this many envs x 256 frames via dd_rollout) at N=1 "
                        "and report it as rollout_point (0 = skip)")
    p.add_argument("--no-extra-points", dest="extra_points", action="store_false",
                   help="skip the notebook-reward point")
    p.add_argument("--gather-point", action="store_true",
                   help="initialise the process group and time gather_point even at N=1 (RCCL at world size "
                        "1 with --dist-backend nccl: the N>1 code path on a one-GPU box)")
    p.add_argument("--hbm-point", type=int, default=16_777_216,
                   help="also time this many drones (HBM-resident) at N=1 and report it as hbm_point (0 = skip)")
    return p.parse_args()


# ----------------------------------------------------------------- CPU baseline
def _cgroup_quota(root: str = "/sys/fs/cgroup", proc: str = "/proc/self/cgroup"):
    """(cpus, file) from this process's cgroup CPU quota, or (None, why not).
    cgroup v2: <root>/<path>/cpu.max = "<quota> <period>" ("max" = none);
    cgroup v1: cpu.cfs_quota_us / cpu.cfs_period_us (quota -1 = none).  The
    process's own cgroup directory is tried first, then the mount root (a
    container's namespace root)."""
    try:
        lines = open(proc).read().split("\n")
    except OSError as e:
        return None, f"{proc}: {e.strerror}"
    v2 = [l.split(":", 2)[2] for l in lines if l.startswith("0::")]
    v1 = [l.split(":", 2)[2] for l in lines if l.count(":") >= 2 and "cpu" in l.split(":", 2)[1].split(",")]
    cands = []
    for rel in v2:
        cands += [("v2", os.path.join(root, rel.lstrip("/")))]
    for rel in v1:
        for mnt in ("cpu", "cpu,cpuacct", "cpuacct,cpu"):
            cands += [("v1", os.path.join(root, mnt, rel.lstrip("/"))), ("v1", os.path.join(root, mnt))]
    cands += [("v2", root)]
    seen = []
    for kind, d in cands:
        try:
            if kind == "v2":
                f = os.path.join(d, "cpu.max")
                quota, period = open(f).read().split()[:2]
                seen.append(f)
                if quota != "max":
                    return float(quota) / float(period), f
            else:
                f = os.path.join(d, "cpu.cfs_quota_us")
                quota = int(open(f).read())
                period = int(open(os.path.join(d, "cpu.cfs_period_us")).read())
                seen.append(f)
                if quota > 0:
                    return quota / period, f
        except (OSError, ValueError):
            continue
    return None, ("no CPU quota set (" + ", ".join(seen) + ")") if seen else "no cgroup CPU controller file readable"


def host_cpu_share() -> dict:
    """The CPUs the CPU baseline may use on this host, with the evidence
    (the reference loop on the host's cores).  In order:
    the cgroup CPU quota (quota / period, rounded down) when one is set;
    otherwise the pool's declared per-job share, OMP_NUM_THREADS / MAX_JOBS
    (the one-GPU box exports 16 and its operators ask worker pools to
    follow it, since os.cpu_count() and the affinity show the whole host);
    otherwise the CPUs in this process's affinity.  Never more than the
    affinity."""
    aff = len(os.sched_getaffinity(0))
    quota, qsrc = _cgroup_quota()
    env = {k: os.environ[k] for k in ("OMP_NUM_THREADS", "MAX_JOBS") if os.environ.get(k, "").isdigit()}
    if quota is not None:
        cores, src = max(1, int(quota)), f"cgroup quota {quota:g} CPUs ({qsrc})"
    elif env:
        k = min(env, key=lambda k: int(env[k]))
        cores, src = int(env[k]), f"{k}={env[k]} (the job's declared CPU share; {qsrc})"
    else:
        cores, src = aff, f"sched_getaffinity ({qsrc})"
    return {"cores": max(1, min(cores, aff)), "source": src, "cgroup_quota_cpus": quota,
            "affinity_cores": aff, "host_cores": os.cpu_count(), "env": env}


def _cpu_worker(args):
    leg, lane0, lanes, steps, seed = args
    from delivery_drone_amd.config import EnvConfig
    from oracle import oracle as ora
    from oracle import pyloop
    t0 = time.perf_counter()
    if leg == "python_objects":
        _, chk = pyloop.bench(lane0, lanes, steps, seed)
    else:
        cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=seed)
        chk = ora.bench(cfg, lane0, lanes, steps)
    return time.perf_counter() - t0, chk


def _cpu_leg(leg: str, seconds: float, workers: int, seed: int, lanes: int, calib_steps: int) -> dict:
    dt, _ = _cpu_worker((leg, 0, lanes, calib_steps, seed))
    per_lane_step = dt / (lanes * calib_steps)
    steps = max(1, int(seconds / (per_lane_step * lanes)))
    ctx = mp.get_context("fork")  # before any GPU call in this process
    jobs = [(leg, w * lanes, lanes, steps, seed) for w in range(workers)]
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        res = pool.map(_cpu_worker, jobs)
    wall = time.perf_counter() - t0
    if not all(math.isfinite(c) for _, c in res):
        raise RuntimeError(f"CPU baseline leg {leg} produced a non-finite checksum")
    total = workers * lanes * steps
    return {"value": round(total / wall, 1), "per_core": round(total / wall / workers, 1),
            "single_process": round(1.0 / per_lane_step, 1), "workers": workers, "drones_per_worker": lanes,
            "frames": steps, "drone_steps": total, "wall_s": round(wall, 2)}


def cpu_baseline(seconds: float, workers: int, seed: int, share: dict | None = None) -> dict:
    """The reference's step on the host's cores, config-3 workload (random
    spawn, auto-reset, uniform random actions, observation every frame), a
    bounded sample of ~`seconds` per leg:

    * python_objects (the value): oracle/pyloop.py, one Python game object
      per drone shaped like DroneGame.step (game_engine.py:95-138) with numpy
      scalar trig and pow squares, pinned bit for bit to the reference's
      fixtures (tests/test_pyloop.py) — the reference loop's own speed;
    * c_scalar: oracle/drone_oracle.c, the fixture-pinned scalar f64 C
      restatement (what a native CPU port reaches).

    `workers` processes per leg (default: host_cpu_share(), recorded with its
    evidence as `cpu_share`; --cpu-workers overrides).  `value` is the
    python_objects leg (`baseline_leg`); `speedup_basis` lists both legs so a
    ratio against either stays comparable across rounds."""
    from oracle import oracle as ora
    ora.build()
    legs = {"python_objects": _cpu_leg("python_objects", seconds, workers, seed, 256, 8),
            "c_scalar": _cpu_leg("c_scalar", seconds, workers, seed, 16_384, 20)}
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except (OSError, IndexError):
        model = platform.processor()
    py, c = legs["python_objects"], legs["c_scalar"]
    share = share or host_cpu_share()
    return {
        "value": py["value"],
        "unit": "env-steps/s",
        "cores": workers,
        "kind": "port",
        "baseline_leg": "python_objects",
        "speedup_basis": {"python_objects": py["value"], "c_scalar": c["value"]},
        "host_cores": os.cpu_count(),
        "affinity_cores": len(os.sched_getaffinity(0)),
        "cpu_share": share,
        "cpu_model": model,
        "cores_note": (f"workers = {workers}: " + (f"the CPU share, {share['source']}" if workers == share["cores"]
                       else "--cpu-workers") + "; per_core is the leg's value / workers"),
        "legs": legs,
        "sample": (f"config-3 workload, {workers} processes per leg on {model} (host: {os.cpu_count()} CPUs, "
                   f"{len(os.sched_getaffinity(0))} in this process's affinity). value = python_objects: "
                   f"oracle/pyloop.py (DroneGame.step-shaped Python objects, fixture-pinned), {py['drone_steps']:.3g} "
                   f"drone-steps in {py['wall_s']} s, {py['per_core']:.3g} per core; c_scalar: "
                   f"oracle/drone_oracle.c, {c['drone_steps']:.3g} drone-steps in {c['wall_s']} s, "
                   f"{c['per_core']:.3g} per core"),
    }


# ------------------------------------------------------------------- GPU bench
class KernelSpanStamps:
    """GPU wall-clock stamps around the timed step kernels.  A one-lane kernel
    (dd_stamp, s_memrealtime at the GPU's constant wall-clock rate) is
    captured at the head of the first timed hipGraph and one at the tail of
    the last, so the stamps bracket the K step kernels and not the host's
    graph submission before the first one.  They replaced
    event-record nodes added to the graph after capture: a graph holding
    those launched ~50 us slower from the host at K = 20 and the wall clock
    paid for it (tools/lab/launch_probe.py, profiles/r06/lab/).  Slots 2 and
    3 are for the calibration graph of the two stamps alone."""

    def __init__(self, lib, dev):
        import ctypes
        import torch
        self.c, self.lib = ctypes, lib
        self.slots = torch.zeros(4, dtype=torch.int64, device=dev)
        khz = ctypes.c_int(0)
        rc = lib.dd_wall_clock_khz(ctypes.byref(khz))
        if rc != 0 or khz.value <= 0:
            raise RuntimeError(f"dd_wall_clock_khz failed: rc {rc}, {khz.value} kHz")
        self.khz = khz.value

    def stamp(self, slot: int, stream) -> None:
        """Launch the stamp kernel for `slot` on `stream` (captured when the stream is capturing)."""
        rc = self.lib.dd_stamp(self.c.c_void_p(self.slots.data_ptr() + 8 * slot), self.c.c_void_p(stream.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"dd_stamp failed: rc {rc}")

    def elapsed_ms(self, first: int = 0, last: int = 1) -> float:
        """Milliseconds between two stamps (synchronises the device)."""
        import torch
        torch.cuda.synchronize(self.slots.device)
        v = self.slots.cpu().tolist()
        return (v[last] - v[first]) / self.khz


def time_steps(env, rows, steps, graph_steps, stream, write_obs=True):
    """Replay `steps` frames from a hipGraph of `graph_steps` launches; returns
    device ms per step (HIP events on the replay stream)."""
    import torch
    nrows = rows.shape[0]
    with torch.cuda.stream(stream):
        for k in range(3):
            env.step(rows[k % nrows], write_obs=write_obs)
        torch.cuda.synchronize(env.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for k in range(graph_steps):
                env.step(rows[k % nrows], write_obs=write_obs)
        g.replay()
        torch.cuda.synchronize(env.device)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        reps = max(1, steps // graph_steps)
        e0.record(stream)
        for _ in range(reps):
            g.replay()
        e1.record(stream)
        torch.cuda.synchronize(env.device)
    return e0.elapsed_time(e1) / (reps * graph_steps)


def hbm_point(n, precision, seed, dev, write_obs, allocs=3, rounds=6, contiguous_allocs=2):
    """The same step at an HBM-resident batch (state + obs >> 256 MiB MALL):
    the roofline the config-3 batch cannot show because it lives in cache.

    At this size the step's time depends on where the driver places the
    arrays physically (identical envs in one process run
    405-490 us; the first allocated is usually the slow one, and which one is
    slow does not follow their virtual offsets).  So `allocs` identical envs
    are allocated one after another and timed in interleaved rounds (order
    reversed every round); every allocation's time is reported, in allocation
    order, and the point's value is their median — the placement spread is
    shown, not picked from.  `contiguous_allocs` more envs with
    memory="contiguous" (one physically contiguous range each) are timed in
    the same rounds and reported beside them (`placements.contiguous`)."""
    import statistics
    import torch
    from delivery_drone_amd import EnvConfig, VecDroneEnv, abi
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=seed)
    rows = torch.randint(0, 8, (4, n), device=dev, dtype=torch.uint8)
    stream = torch.cuda.Stream(dev)
    graph_steps = 10
    runs = []
    for j in range(max(1, allocs) + max(0, contiguous_allocs)):
        mem = "torch" if j < max(1, allocs) else "contiguous"
        env = VecDroneEnv(n, device=dev, config=cfg, precision=precision, memory=mem)
        env.reset()
        with torch.cuda.stream(stream):
            for k in range(3):
                env.step(rows[k % 4], write_obs=write_obs)
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                for k in range(graph_steps):
                    env.step(rows[k % 4], write_obs=write_obs)
            g.replay()
        torch.cuda.synchronize(dev)
        runs.append((env, g, []))
    for rnd in range(rounds):
        for env, g, ts in (runs if rnd % 2 == 0 else runs[::-1]):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(stream):
                e0.record(stream)
                for _ in range(2):
                    g.replay()
                e1.record(stream)
            torch.cuda.synchronize(dev)
            ts.append(e0.elapsed_time(e1) / (2 * graph_steps))
    bpe = runs[0][0].step_bytes_per_env(abi.DD_ACT_BITMASK, with_obs=write_obs)
    contig = [statistics.median(ts) for env, _, ts in runs if env.memory == "contiguous"]
    per_alloc = [statistics.median(ts) for env, _, ts in runs if env.memory == "torch"]
    ms = statistics.median(per_alloc)
    gbs = bpe * n / (ms * 1e-3) / 1e9
    out = {"envs": n, "us_per_step": round(ms * 1e3, 3), "steps_per_s": round(n / (ms * 1e-3), 1),
           "achieved": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
           "placements": {"allocations": len(per_alloc), "us_per_step_by_allocation": [round(t * 1e3, 1) for t in per_alloc],
                          "frac_by_allocation": [round(bpe * n / (t * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                                 for t in per_alloc],
                          "frac_min": round(bpe * n / (max(per_alloc) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                          "frac_max": round(bpe * n / (min(per_alloc) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                          "value": "median over allocations",
                          "contiguous": {"allocations": len(contig),
                                         "us_per_step_by_allocation": [round(t * 1e3, 1) for t in contig],
                                         "frac_by_allocation": [round(bpe * n / (t * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                                                for t in contig],
                                         "note": "VecDroneEnv(memory='contiguous'): every field in one "
                                                 "physically contiguous range, timed in the same rounds"}},
           "traffic": pmc_traffic(n, precision, write_obs), "bytes_per_env": bpe}
    del runs, rows
    torch.cuda.empty_cache()
    return out


def rollout_point(n, frames, precision, seed, dev, warm=120, timed=40):
    """BASELINE config 5, the PPO rollout shape: n envs x `frames` frames,
    reward + done fused into the step kernel, obs written into a
    [frames, n, 15] rollout buffer — one dd_rollout launch per rollout, actions
    read from a resident [frames, n] buffer.  Bytes per env-frame: action 1 +
    reward 4 + done 1 + obs 60 (state in/out once per rollout).

    Timing: a launch costs a constant ~560k shader cycles, and
    its time follows the clock the chip holds.  Back-to-back launches see a
    DVFS transient (GRBM_GUI_ACTIVE per dispatch, profiles/r05/c5_dvfs/): the
    effective clock falls from ~2.23 to ~1.93 GHz a few launches in and comes
    back to ~2.28 GHz after ~25 ms of sustained load.  So `warm` untimed
    launches run first and `timed` launches are timed one by one (HIP events
    on the launch stream): ms_per_rollout is their median (the steady state);
    the first launches and the transient's worst are reported beside it."""
    import statistics
    import torch
    from delivery_drone_amd import EnvConfig, VecDroneEnv
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=seed)
    env = VecDroneEnv(n, device=dev, config=cfg, precision=precision)
    env.reset()
    acts = torch.randint(0, 8, (frames, n), device=dev, dtype=torch.uint8)
    obs = torch.empty(frames, n, 15, device=dev)
    rew = torch.empty(frames, n, device=dev, dtype=env.float_dtype)
    done = torch.empty(frames, n, device=dev, dtype=torch.bool)
    stream = torch.cuda.Stream(dev)
    total_launches = warm + timed
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * total_launches)]
    with torch.cuda.stream(stream):
        env.rollout(acts, obs_out=obs, reward_out=rew, done_out=done)  # first launch: code objects, LDS set-up
        torch.cuda.synchronize(dev)
        for k in range(total_launches):
            ev[2 * k].record(stream)
            env.rollout(acts, obs_out=obs, reward_out=rew, done_out=done)
            ev[2 * k + 1].record(stream)
        torch.cuda.synchronize(dev)
    env.check_device_errors()
    ms_all = [ev[2 * k].elapsed_time(ev[2 * k + 1]) for k in range(total_launches)]
    steady = ms_all[warm:]
    ms = statistics.median(steady)
    fbytes = 1 + rew.element_size() + 1 + 60
    state = env.step_bytes_per_env(with_obs=False) - 1 - rew.element_size() - 1  # state read + write once
    total = n * frames * fbytes + n * state
    gbs = total / (ms * 1e-3) / 1e9
    traffic, traffic_note = pmc_traffic_row(n, precision, True, kernel="rollout_kernel", frames=frames)
    out = {"envs": n, "frames": frames, "ms_per_rollout": round(ms, 4),
           "steps_per_s": round(n * frames / (ms * 1e-3), 1), "achieved": round(gbs, 1),
           "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_env_frame": fbytes, "bytes_per_launch": total,
           "timing": {"warm_launches": warm, "timed_launches": timed,
                      "ms_steady_median": round(ms, 4), "ms_steady_mean": round(statistics.mean(steady), 4),
                      "ms_all_mean": round(statistics.mean(ms_all), 4),
                      "frac_all_mean": round(total / (statistics.mean(ms_all) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                      "ms_first5_median": round(statistics.median(ms_all[:5]), 4),
                      "ms_transient_max": round(max(ms_all[:warm]), 4),
                      "rule": "median of the timed launches after the warm ones (DVFS transient excluded)"},
           "kernel_choice": env.last_rollout_kernel,
           "traffic": traffic, "traffic_note": traffic_note,
           "kernel": "dd::rollout_kernel (dd_rollout, one launch per 256-frame rollout)"}
    del env, acts, obs, rew, done
    torch.cuda.empty_cache()
    return out


def step_loop_point(n, frames, precision, seed, dev):
    """BASELINE config 5 variant (a): the same rollout as one dd_step launch
    per frame (actions from a [frames, n] tensor, obs/reward/done written
    straight into the rollout buffers with step(out=...)), the frames
    captured in one hipGraph.  Per frame the state makes a full HBM round
    trip, so bytes per env-frame are the step's 147 (f32, with obs)."""
    import torch
    from delivery_drone_amd import EnvConfig, VecDroneEnv, abi
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=seed)
    env = VecDroneEnv(n, device=dev, config=cfg, precision=precision)
    env.reset()
    acts = torch.randint(0, 8, (frames, n), device=dev, dtype=torch.uint8)
    obs = torch.empty(frames, n, 15, device=dev)
    rew = torch.empty(frames, n, device=dev, dtype=env.float_dtype)
    done = torch.empty(frames, n, device=dev, dtype=torch.bool)
    stream = torch.cuda.Stream(dev)
    with torch.cuda.stream(stream):
        for t in range(3):
            env.step(acts[t], out=(obs[t], rew[t], done[t]))
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for t in range(frames):
                env.step(acts[t], out=(obs[t], rew[t], done[t]))
        g.replay()
        torch.cuda.synchronize(dev)
        reps = 5
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            g.replay()
        e1.record(stream)
        torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    bpe = env.step_bytes_per_env(abi.DD_ACT_BITMASK, with_obs=True)
    gbs = bpe * n * frames / (ms * 1e-3) / 1e9
    del env, acts, obs, rew, done, g
    torch.cuda.empty_cache()
    return {"envs": n, "frames": frames, "ms_per_rollout": round(ms, 4),
            "steps_per_s": round(n * frames / (ms * 1e-3), 1), "us_per_frame": round(ms * 1e3 / frames, 3),
            "achieved": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_env_frame": bpe,
            "launch": f"hipGraph of {frames} dd_step launches into [T, N] buffers"}


def config2_point(seed, dev, n=4096):
    """BASELINE config 2: 4096 drones, fixed spawn (drone 400,100; pad
    400,500), f32 storage, auto-reset.  Launch-bound: one dd_step per frame
    from a hipGraph, and the same frames as 256-frame dd_rollout launches."""
    import torch
    from delivery_drone_amd import EnvConfig, VecDroneEnv
    cfg = EnvConfig(randomize_drone=False, randomize_platform=False, auto_reset=True, seed=seed)
    env = VecDroneEnv(n, device=dev, config=cfg)
    env.reset()
    rows = torch.randint(0, 8, (8, n), device=dev, dtype=torch.uint8)
    ms = time_steps(env, rows, 2000, 100, torch.cuda.Stream(dev))
    frames = 256
    acts = torch.randint(0, 8, (frames, n), device=dev, dtype=torch.uint8)
    obs = torch.empty(frames, n, 15, device=dev)
    rew = torch.empty(frames, n, device=dev)
    done = torch.empty(frames, n, device=dev, dtype=torch.bool)
    stream = torch.cuda.Stream(dev)
    with torch.cuda.stream(stream):
        env.rollout(acts, obs_out=obs, reward_out=rew, done_out=done)
        torch.cuda.synchronize(dev)
        reps = 20
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            env.rollout(acts, obs_out=obs, reward_out=rew, done_out=done)
        e1.record(stream)
        torch.cuda.synchronize(dev)
    rms = e0.elapsed_time(e1) / reps
    del env, rows, acts, obs, rew, done
    torch.cuda.empty_cache()
    return {"envs": n, "spawn": "fixed", "us_per_step": round(ms * 1e3, 3),
            "steps_per_s": round(n / (ms * 1e-3), 1), "launch": "hipGraph of 100 dd_step",
            "rollout_ms_per_256_frames": round(rms, 4),
            "rollout_steps_per_s": round(n * frames / (rms * 1e-3), 1)}


def _sync(dev):
    import torch
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def gather_point(obs, n, world, backend, reps=5):
    """BASELINE config 4's optional exchange: every rank's obs block [n, 15]
    gathered to rank 0 (sharding.gather_obs: RCCL gather over xGMI with
    backend nccl; gloo moves host copies), timed outside the step loop.
    Collective: every rank calls it.  Rank 0 checks the gathered shape and
    that its own block arrived unchanged (tests/test_bench_contract.py runs
    this on gloo ranks)."""
    import torch
    import torch.distributed as dist
    from delivery_drone_amd.sharding import gather_obs
    dev = obs.device
    obs = obs if backend == "nccl" else obs.cpu()
    gather_obs(obs, n * world)  # warm-up (communicator set-up)
    _sync(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = gather_obs(obs, n * world)
    _sync(dev)
    dt = (time.perf_counter() - t0) / reps
    dt = reduce_max([dt], backend, dev)[0]
    if dist.get_rank() == 0:
        if tuple(out.shape) != (n * world, obs.shape[1]) or not torch.equal(out[:n], obs):
            raise RuntimeError(f"gather_obs returned {tuple(out.shape)} / a changed rank-0 block")
    nbytes = n * world * 15 * 4
    del out
    return {"rows": n * world, "bytes_to_rank0": nbytes, "ms": round(dt * 1e3, 3),
            "GB_per_s": round(nbytes / dt / 1e9, 2), "backend": backend,
            "note": "timed outside the step loop; the step path has no collective"}


def reduce_max(values, backend, dev):
    """Element-wise max of `values` over all ranks (the bench's timing rule:
    the slowest rank's wall and device time)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(values, dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t]


def f64_point(n, seed, dev, steps=500, graph_steps=50):
    """The headline workload (config 3: n drones, random spawn, auto-reset,
    obs every frame) with the state stored at the reference's own width
    (precision='f64', Python floats: drone.py:12-42): same arithmetic, 80 B
    of state per drone instead of 40, bytes per env from
    dd_step_bytes_per_env(DD_F64, ...)."""
    import torch
    from delivery_drone_amd import EnvConfig, VecDroneEnv, abi
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=seed)
    env = VecDroneEnv(n, device=dev, config=cfg, precision="f64")
    env.reset()
    rows = torch.randint(0, 8, (8, n), device=dev, dtype=torch.uint8)
    ms = time_steps(env, rows, steps, graph_steps, torch.cuda.Stream(dev))
    bpe = env.step_bytes_per_env(abi.DD_ACT_BITMASK, with_obs=True)
    assert bpe == abi.lib().dd_step_bytes_per_env(abi.DD_F64, abi.DD_ACT_BITMASK, 1)
    gbs = bpe * n / (ms * 1e-3) / 1e9
    del env, rows
    torch.cuda.empty_cache()
    return {"envs": n, "precision": "f64", "us_per_step": round(ms * 1e3, 3), "steps_per_s": round(n / (ms * 1e-3), 1),
            "achieved": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_env": bpe,
            "kernel": "dd::step_kernel<double, 0, true, false>", "launch": f"hipGraph of {graph_steps} dd_step"}


def ping_pong_point(n, seed, dev, steps=2000, graph_steps=50, rounds=3):
    """The headline workload with VecDroneEnv(ping_pong=True) (DDStepIO.state_out:
    the nine per-frame fields read from one copy and written to the other)
    timed against in-place stepping of an identical env, interleaved rounds on
    one box; the same bytes per env either way (each field is read once and
    written once per step).  Graphs hold an even number of steps."""
    import statistics
    import torch
    from delivery_drone_amd import EnvConfig, VecDroneEnv, abi
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=seed)
    envs = {m: VecDroneEnv(n, device=dev, config=cfg, ping_pong=(m == "ping_pong")) for m in ("in_place", "ping_pong")}
    rows = torch.randint(0, 8, (8, n), device=dev, dtype=torch.uint8)
    ts = {m: [] for m in envs}
    for e in envs.values():
        e.reset()
    for r in range(rounds):
        for m in (list(envs) if r % 2 == 0 else list(envs)[::-1]):
            ts[m].append(time_steps(envs[m], rows, steps, graph_steps, torch.cuda.Stream(dev)))
    bpe = envs["in_place"].step_bytes_per_env(abi.DD_ACT_BITMASK, with_obs=True)
    out = {"envs": n, "bytes_per_env": bpe, "launch": f"hipGraph of {graph_steps} dd_step", "rounds": rounds}
    for m, t in ts.items():
        ms = statistics.median(t)
        gbs = bpe * n / (ms * 1e-3) / 1e9
        out[m] = {"us_per_step": round(ms * 1e3, 3), "us_by_round": [round(x * 1e3, 3) for x in t],
                  "steps_per_s": round(n / (ms * 1e-3), 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}
    del envs, rows
    torch.cuda.empty_cache()
    return out


def gae_point(n, frames, dev):
    """dd_gae over a [frames, n] rollout: reads reward,
    value (+ bootstrap row), done; writes advantage and return."""
    import torch
    from delivery_drone_amd import gae
    rew = torch.randn(frames, n, device=dev)
    val = torch.randn(frames + 1, n, device=dev)
    done = torch.rand(frames, n, device=dev) < 0.01
    adv = torch.empty(frames, n, device=dev)
    ret = torch.empty(frames, n, device=dev)
    stream = torch.cuda.Stream(dev)
    with torch.cuda.stream(stream):
        gae(rew, val, done, out=(adv, ret))
        torch.cuda.synchronize(dev)
        reps = 20
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            gae(rew, val, done, out=(adv, ret))
        e1.record(stream)
        torch.cuda.synchronize(dev)
    us = e0.elapsed_time(e1) * 1e3 / reps
    nbytes = frames * n * (4 + 4 + 1 + 4 + 4) + n * 4
    gbs = nbytes / (us * 1e-6) / 1e9
    del rew, val, done, adv, ret
    torch.cuda.empty_cache()
    return {"envs": n, "frames": frames, "us": round(us, 2), "achieved": round(gbs, 1),
            "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes": nbytes, "kernel": "dd::gae_kernel"}


def notebook_point(n, precision, seed, dev, mode="notebook"):
    """The step with a notebook's reward fused:
    reward_mode='notebook' (PPO's calc_reward with its two-frame history) or
    'reinforce' (Policy_Gradients.ipynb's), max_steps=300, config-3 batch."""
    import torch
    from delivery_drone_amd import EnvConfig, VecDroneEnv, abi
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=seed)
    env = VecDroneEnv(n, device=dev, config=cfg, precision=precision, reward_mode=mode, max_steps=300)
    env.reset()
    rows = torch.randint(0, 8, (8, n), device=dev, dtype=torch.uint8)
    ms = time_steps(env, rows, 500, 50, torch.cuda.Stream(dev))
    fb = 4 if precision == "f32" else 8
    # + shaped reward and done; PPO also reads and writes its f64 history slot
    bpe = env.step_bytes_per_env(abi.DD_ACT_BITMASK, with_obs=True) + fb + 1 + (16 if mode == "notebook" else 0)
    gbs = bpe * n / (ms * 1e-3) / 1e9
    del env, rows
    torch.cuda.empty_cache()
    return {"envs": n, "us_per_step": round(ms * 1e3, 3), "steps_per_s": round(n / (ms * 1e-3), 1),
            "achieved": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_env": bpe,
            "kernel": f"dd::step_kernel<float, 0, true, {1 if mode == 'notebook' else 2}> (reward_mode='{mode}')"}


MLP_FLOPS_PER_ROW = 2 * (15 * 128 + 128 * 128 + 128 * 64 + 64 * 3)  # the notebooks' actor, algorithmic
F32_MFMA_PEAK_TFS = 157.3  # MI355X dense f32 MFMA (MI355X_MICROARCH.md, Matrix cores)
F16_MFMA_PEAK_TFS = 2516.6  # dense f16 MFMA, ~2.5 PF (MI355X_MICROARCH.md: 32x32x16 at 32 cycles/SIMD, 2.4 GHz)


def _random_actor(dev, seed, compute="f32"):
    """The notebooks' DroneGamerBoi body with torch's default init (random
    weights of that architecture; no checkpoint travels to the box)."""
    import torch
    from torch import nn
    from delivery_drone_amd import MlpNet
    torch.manual_seed(seed)
    net = nn.Sequential(nn.Linear(15, 128), nn.LayerNorm(128), nn.ReLU(), nn.Linear(128, 128), nn.LayerNorm(128),
                        nn.ReLU(), nn.Linear(128, 64), nn.LayerNorm(64), nn.ReLU(), nn.Linear(64, 3))
    return MlpNet(net.state_dict(), device=dev, compute=compute)


def policy_point(n, seed, dev, compute="f32"):
    """the actor forward + Bernoulli sample + log-prob
    (dd_mlp_forward) over n observation rows; bound = the MFMA of `compute`
    (f32: 157.3 TF dense; f16x3: three f16 MFMAs per product, priced against
    the f16 MFMA's 2.5 PF at 3x the algorithmic flops)."""
    import torch
    actor = _random_actor(dev, seed, compute)
    obs = torch.randn(n, 15, device=dev)
    acts = torch.empty(n, dtype=torch.uint8, device=dev)
    lp = torch.empty(n, device=dev)
    stream = torch.cuda.Stream(dev)
    with torch.cuda.stream(stream):
        actor.act(obs, actions_out=acts, log_prob_out=lp)
        torch.cuda.synchronize(dev)
        reps = 50  # one hipGraph of 50 launches: device time, no host gaps between them
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for s in range(reps):
                actor.act(obs, step=s, actions_out=acts, log_prob_out=lp)
        g.replay()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(4):
            g.replay()
        e1.record(stream)
        torch.cuda.synchronize(dev)
    us = e0.elapsed_time(e1) * 1e3 / (4 * reps)
    tfs = n * MLP_FLOPS_PER_ROW / (us * 1e-6) / 1e12
    del actor, obs, acts, lp, g
    torch.cuda.empty_cache()
    if compute == "f32":
        roof = {"bound": "mfma", "achieved": round(tfs, 2), "peak": F32_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                "frac": round(tfs / F32_MFMA_PEAK_TFS, 4), "flops_per_row": MLP_FLOPS_PER_ROW}
        kernel = "dd::mlp::mlp_kernel<3, false> (dd_mlp_forward: actor + Bernoulli sample + log-prob, f32 MFMA)"
    else:  # the MFMA pipe runs 3x the algorithmic flops (hi.hi, hi.lo, lo.hi)
        roof = {"bound": "mfma", "achieved": round(3 * tfs, 2), "peak": F16_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                "frac": round(3 * tfs / F16_MFMA_PEAK_TFS, 4), "flops_per_row": 3 * MLP_FLOPS_PER_ROW,
                "algorithmic_tflops": round(tfs, 2), "algorithmic_frac": round(tfs / F16_MFMA_PEAK_TFS, 4),
                "frac_note": "frac prices the pipe's work (3 f16 products per product); algorithmic_frac the "
                             "network's own flops against the same f16 peak"}
        kernel = "dd::mlp::mlp_kernel<3, true> (dd_mlp_forward, DD_MLP_F16X3: split f16 operands on the f16 MFMA)"
    return {"rows": n, "compute": compute, "us": round(us, 2), "launch": "hipGraph of 50 dd_mlp_forward",
            "rows_per_s": round(n / (us * 1e-6), 1), "roofline": roof, "kernel": kernel}


def policy_rollout_point(n, frames, seed, dev, compute="f32"):
    """Policy in the loop, nothing on the host: per frame dd_mlp_forward
    (sample from the current obs) then dd_step, `frames` frames captured in
    one hipGraph.  env-steps/s with the actor's inference included."""
    import torch
    from delivery_drone_amd import EnvConfig, VecDroneEnv
    actor = _random_actor(dev, seed, compute)
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=seed)
    env = VecDroneEnv(n, device=dev, config=cfg)
    obs = env.reset()
    acts = torch.empty(n, dtype=torch.uint8, device=dev)
    lp = torch.empty(n, device=dev)
    stream = torch.cuda.Stream(dev)
    with torch.cuda.stream(stream):
        for t in range(3):
            actor.act(obs, step=t, actions_out=acts, log_prob_out=lp)
            env.step(acts)
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for t in range(frames):
                actor.act(env.obs, step=t, actions_out=acts, log_prob_out=lp)
                env.step(acts)
        g.replay()
        torch.cuda.synchronize(dev)
        reps = 5
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            g.replay()
        e1.record(stream)
        torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    del actor, env, acts, lp, g
    torch.cuda.empty_cache()
    return {"envs": n, "frames": frames, "compute": compute, "ms": round(ms, 3),
            "steps_per_s": round(n * frames / (ms * 1e-3), 1), "us_per_frame": round(ms * 1e3 / frames, 2),
            "launch": f"hipGraph of {frames} x (dd_mlp_forward + dd_step)"}


def policy_fused_point(n, frames, seed, dev, compute="f16x3", reps=5):
    """collect_episodes_ppo with the actor in the loop as ONE launch
    (dd_policy_rollout, VecDroneEnv.policy_rollout): per frame the actor,
    Bernoulli sampling and the frame, writing the PPO buffers obs [T, N, 15],
    actions, log-probs, rewards and dones.  env-steps/s with the policy's
    inference included; same work as policy_rollout_point plus the per-frame
    buffers that point does not keep."""
    import torch
    from delivery_drone_amd import EnvConfig, VecDroneEnv
    actor = _random_actor(dev, seed, compute)
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=seed)
    env = VecDroneEnv(n, device=dev, config=cfg)
    env.reset()
    bufs = dict(obs_out=torch.empty(frames, n, 15, device=dev),
                actions_out=torch.empty(frames, n, dtype=torch.uint8, device=dev),
                log_prob_out=torch.empty(frames, n, device=dev), reward_out=torch.empty(frames, n, device=dev),
                done_out=torch.empty(frames, n, dtype=torch.bool, device=dev))
    stream = torch.cuda.Stream(dev)
    with torch.cuda.stream(stream):
        env.policy_rollout(actor, frames, seed=seed, **bufs)  # warm-up (and LDS attribute set-up)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for r in range(reps):
            env.policy_rollout(actor, frames, seed=seed, step=(r + 1) * frames, **bufs)
        e1.record(stream)
        torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    tfs = n * frames * MLP_FLOPS_PER_ROW / (ms * 1e-3) / 1e12
    del actor, env, bufs
    torch.cuda.empty_cache()
    if compute == "f32":
        roof = {"bound": "mfma", "achieved": round(tfs, 2), "peak": F32_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                "frac": round(tfs / F32_MFMA_PEAK_TFS, 4), "flops_per_drone_frame": MLP_FLOPS_PER_ROW}
    else:  # three f16 MFMAs per product, as policy_point prices them
        roof = {"bound": "mfma", "achieved": round(3 * tfs, 2), "peak": F16_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                "frac": round(3 * tfs / F16_MFMA_PEAK_TFS, 4), "flops_per_drone_frame": 3 * MLP_FLOPS_PER_ROW,
                "algorithmic_tflops": round(tfs, 2), "algorithmic_frac": round(tfs / F16_MFMA_PEAK_TFS, 4),
                "frac_note": "frac prices the pipe's work (3 f16 products per product); algorithmic_frac the "
                             "network's own flops against the same f16 peak"}
    return {"envs": n, "frames": frames, "compute": compute, "ms": round(ms, 3),
            "steps_per_s": round(n * frames / (ms * 1e-3), 1), "us_per_frame": round(ms * 1e3 / frames, 2),
            "roofline": roof, "launch": f"one dd_policy_rollout launch per {frames} frames",
            "kernel": f"dd::prl::policy_rollout_kernel<float, {'true' if compute == 'f16x3' else 'false'}, true>"}


def render_point(seed, dev, frames=64, reps=20):
    """DroneGame.render('rgb_array') as dd_render, `frames`
    lanes of a running batch per launch (HUD and game-over overlay on).
    Bound by the frame bytes it writes: 800 x 600 x 3 per frame."""
    import torch
    from delivery_drone_amd import EnvConfig, VecDroneEnv
    env = VecDroneEnv(4096, device=dev, config=EnvConfig(randomize_drone=True, auto_reset=True, seed=seed))
    env.reset()
    acts = torch.randint(0, 8, (4096,), device=dev, dtype=torch.uint8)
    for _ in range(40):
        env.step(acts)
    lanes = torch.arange(0, 4096, 4096 // frames, dtype=torch.int32, device=dev)[:frames]
    out = torch.empty(frames, 600, 800, 3, dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(dev)
    with torch.cuda.stream(stream):
        env.render(lanes=lanes, out=out)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            env.render(lanes=lanes, out=out)
        e1.record(stream)
        torch.cuda.synchronize(dev)
    us = e0.elapsed_time(e1) * 1e3 / reps
    nbytes = frames * 600 * 800 * 3
    gbs = nbytes / (us * 1e-6) / 1e9
    res = {"frames": frames, "us": round(us, 2), "frames_per_s": round(frames / (us * 1e-6), 1),
           "achieved": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes": nbytes,
           "kernel": "dd::render::render_kernel (dd_render, rgb_array 800x600, HUD on)"}
    del env, out
    torch.cuda.empty_cache()
    return res


def socket_point(seed, dev, steps=2000):
    """STEP round trips through the JSON-lines socket
    server (reference protocol) from one client on 127.0.0.1, like the
    reference's benchmark_latency (socket_client.py:227-282)."""
    import json as _json
    import socket
    from delivery_drone_amd import VecDroneEnv
    from delivery_drone_amd.server import BatchSocketServer
    env = VecDroneEnv(1, device=dev, auto_reset=False, randomize_drone=True, seed=seed, precision="f64")
    env.reset()
    srv = BatchSocketServer(env, "127.0.0.1", 0).start()
    try:
        sock = socket.create_connection(("127.0.0.1", srv.port), timeout=30)
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        f = sock.makefile("rb")
        f.readline()  # HANDSHAKE
        step = (_json.dumps({"type": "STEP", "game_id": 0, "action": {"main_thrust": 1}}) + "\n").encode()
        reset = (_json.dumps({"type": "RESET", "game_id": 0}) + "\n").encode()

        def run(k):
            for _ in range(k):
                sock.sendall(step)
                if _json.loads(f.readline())["done"]:
                    sock.sendall(reset)
                    f.readline()

        run(50)
        t0 = time.perf_counter()
        run(steps)
        dt = time.perf_counter() - t0
        sock.close()
    finally:
        srv.stop()
    return {"steps": steps, "steps_per_s": round(steps / dt, 1), "ms_per_step": round(dt * 1e3 / steps, 4),
            "transport": "TCP 127.0.0.1, JSON lines, one client, sequential STEP requests",
            "reference_published": "300-500 steps/s (delivery_drone/SOCKET_API.md:373)"}


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """`python bench.py --gpus N` (N > 1) outside torch.distributed.run: this
    process is the launcher, not a rank.  It touches no GPU (a device count
    initialises nothing on this image), runs the CPU baseline once, then starts
    N fresh ranks as a child `torch.distributed.run` (a child process, never an
    exec), hands rank 0 the baseline through a file and relays rank 0's JSON
    line.  Returns the children's exit code."""
    import subprocess
    import tempfile
    if args.dist_backend == "nccl":
        import torch
        ndev = torch.cuda.device_count()
        if ndev < args.gpus:
            raise SystemExit(f"--gpus {args.gpus} with --dist-backend nccl but {ndev} visible GPUs: "
                             "RCCL needs one GPU per rank")
    cpu_file = None
    if args.cpu_baseline > 0:
        share = host_cpu_share()
        cpu = cpu_baseline(args.cpu_baseline, args.cpu_workers or share["cores"], args.seed, share)
        fd, cpu_file = tempfile.mkstemp(prefix="dd_cpu_baseline_", suffix=".json")
        with os.fdopen(fd, "w") as f:
            json.dump(cpu, f)
    argv = [a for a in sys.argv[1:]]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + argv + \
          ["--cpu-baseline", "0"] + (["--cpu-baseline-json", cpu_file] if cpu_file else [])
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", DD_BENCH_LAUNCHER="1")
    try:
        r = subprocess.run(cmd, stdout=subprocess.PIPE, env=env, text=True)
    finally:
        if cpu_file:
            os.unlink(cpu_file)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    for ln in r.stdout.splitlines():
        if not ln.startswith("{"):
            print(ln, file=sys.stderr)
    if r.returncode == 0 and len(lines) != 1:
        print(f"expected one JSON line from rank 0, got {len(lines)}", file=sys.stderr)
        return 1
    for ln in lines:
        print(ln, flush=True)
    return r.returncode


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(launch_ranks(args))
    if world != args.gpus:
        args.gpus = world

    cpu = None
    if rank == 0 and args.cpu_baseline > 0:
        # before any GPU call (the legs fork worker processes); at N > 1 under
        # torch.distributed.run the other ranks wait in the rendezvous meanwhile
        share = host_cpu_share()
        workers = args.cpu_workers or share["cores"]
        cpu = cpu_baseline(args.cpu_baseline, workers, args.seed, share)
    elif rank == 0 and args.cpu_baseline_json:
        with open(args.cpu_baseline_json) as f:
            cpu = json.load(f)
        cpu["measured_by"] = "the launcher process (bench.py --gpus N), before the ranks started"

    import torch
    import torch.distributed as dist

    from delivery_drone_amd import EnvConfig, VecDroneEnv, abi

    ndev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and world > ndev:
        raise SystemExit(f"{world} ranks but {ndev} visible GPUs: RCCL needs one GPU per rank")
    local_dev = local % max(ndev, 1)
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    use_pg = world > 1 or args.gather_point
    if use_pg:
        if "MASTER_ADDR" not in os.environ:  # --gather-point outside torch.distributed.run
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29531"),
                              RANK="0", WORLD_SIZE="1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    n = args.envs_per_gpu
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=args.seed)
    env = VecDroneEnv(n, device=dev, config=cfg, precision=args.precision, env_id_base=rank * n)
    env.reset()
    gen = torch.Generator(device=dev).manual_seed(args.seed * 1000 + rank)
    rows = torch.randint(0, 8, (args.action_rows, n), device=dev, generator=gen, dtype=torch.uint8)
    write_obs = not args.no_obs

    stream = torch.cuda.Stream(dev)
    stream.wait_stream(torch.cuda.current_stream(dev))
    counter = [0]

    def one_step():
        env.step(rows[counter[0] % args.action_rows], write_obs=write_obs)
        counter[0] += 1

    # Timed launches replay from hipGraphs of G = min(--graph-steps, K) steps
    # plus one graph of the K % G remainder, so the timed region has the same
    # shape (graph launches, no per-step host gaps) whatever K is.  (Sizing G
    # to the warmup too, so the warmup replays the timed graph, was slower at
    # K = 20, W = 5: four 5-launch replays leave gaps, profiles/r02/k20.)
    G = min(args.graph_steps, max(args.steps, 1))
    graphs = {}
    # The kernels' own span: GPU wall-clock stamps written by one-lane kernels
    # captured INSIDE the timed graphs (KernelSpanStamps), one at the head of
    # the first graph of the timed region and one at the tail of its last.
    # They bracket the K step kernels only, not the host's graph submission
    # before the first one (at K = 20 that submission gap sat inside the
    # stream events below and priced launch overhead into roofline.frac:
    # VERDICT r05 #1).
    spans = KernelSpanStamps(env._lib, dev)
    seq = ([G] * (args.steps // G) + ([args.steps % G] if args.steps % G else [])) if G > 0 else []
    timed = [(k, j == 0, j == len(seq) - 1) for j, k in enumerate(seq)]

    def graph_of(k: int, head: bool = False, tail: bool = False):
        key = (k, head, tail)
        if key not in graphs:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                if head:
                    spans.stamp(0, stream)
                for i in range(k):
                    env.step(rows[i % args.action_rows], write_obs=write_obs)
                if tail:
                    spans.stamp(1, stream)
            graphs[key] = g
        return graphs[key]

    with torch.cuda.stream(stream):
        if G > 0:
            for _ in range(3):  # settle allocations before capture
                one_step()
            torch.cuda.synchronize(dev)
            for k in {G, args.warmup % G} - {0}:
                graph_of(k)
            for key in set(timed):
                graph_of(*key)

        def run_warmup(k: int):
            if G <= 0:
                for _ in range(k):
                    one_step()
                return
            for _ in range(k // G):
                graphs[(G, False, False)].replay()
            if k % G:
                graphs[(k % G, False, False)].replay()

        def run_timed():
            if G <= 0:
                spans.stamp(0, stream)
                for _ in range(args.steps):
                    one_step()
                spans.stamp(1, stream)
                return
            for key in timed:
                graphs[key].replay()

        run_warmup(args.warmup)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        run_timed()
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
            torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)
    span_ms = spans.elapsed_ms(0, 1)
    # The stamps' own cost (the head stamp's kernel end and the tail stamp's
    # dispatch lie inside the span): an untimed graph of the two stamps
    # alone, replayed after the timed region, measures it and it is
    # subtracted.
    marker_ms = 0.0
    if G > 0:
        import statistics
        gc = torch.cuda.CUDAGraph()
        with torch.cuda.stream(stream), torch.cuda.graph(gc, stream=stream):
            spans.stamp(2, stream)
            spans.stamp(3, stream)
        cals = []
        for _ in range(7):
            gc.replay()
            cals.append(spans.elapsed_ms(2, 3))
        marker_ms = statistics.median(cals)
    kernel_ms = span_ms - marker_ms

    wall, gpu_ms, kernel_ms = reduce_max([wall, gpu_ms, kernel_ms], args.dist_backend, dev)

    # sanity: the batch is alive and finite
    assert torch.isfinite(env.obs).all().item() and int(env.episode.max()) >= 1
    hbm = None
    if world == 1 and args.hbm_point > 0:
        hbm = hbm_point(args.hbm_point, args.precision, args.seed, dev, write_obs)
    gp = None
    if use_pg:
        try:  # an optional extra: a failure here must not cost the step measurement
            gp = gather_point(env.obs, n, world, args.dist_backend)
        except Exception as e:  # noqa: BLE001
            gp = {"error": f"{type(e).__name__}: {e}"[:300]}
    c5 = c5a = g5 = c2 = nb = rf = f64p = ppp = pp = pr = pp16 = pr16 = pf = pf16 = sp = rp = None
    if world == 1 and args.rollout_point > 0:
        c5 = rollout_point(args.rollout_point, 256, args.precision, args.seed, dev)
        c5a = step_loop_point(args.rollout_point, 256, args.precision, args.seed, dev)
        g5 = gae_point(args.rollout_point, 256, dev)
    if world == 1 and args.extra_points:
        c2 = config2_point(args.seed, dev)
        nb = notebook_point(n, args.precision, args.seed, dev)
        rf = notebook_point(n, args.precision, args.seed, dev, "reinforce")
        f64p = f64_point(n, args.seed, dev)
        ppp = ping_pong_point(n, args.seed, dev)
        pp = policy_point(args.rollout_point or 65_536, args.seed, dev)
        pr = policy_rollout_point(args.rollout_point or 65_536, 64, args.seed, dev)
        pp16 = policy_point(args.rollout_point or 65_536, args.seed, dev, "f16x3")
        pr16 = policy_rollout_point(args.rollout_point or 65_536, 64, args.seed, dev, "f16x3")
        pf = policy_fused_point(args.rollout_point or 65_536, 64, args.seed, dev, "f32")
        pf16 = policy_fused_point(args.rollout_point or 65_536, 64, args.seed, dev, "f16x3")
        sp = socket_point(args.seed, dev)
        rp = render_point(args.seed, dev)

    pg_world = dist.get_world_size() if use_pg else 1
    if rank == 0:
        total_steps = n * pg_world * args.steps
        value = total_steps / wall
        step_ms = kernel_ms / args.steps  # the K step kernels' own span per launch
        bytes_env = env.step_bytes_per_env(abi.DD_ACT_BITMASK, with_obs=write_obs)
        traffic, traffic_note = pmc_traffic_row(n, args.precision, write_obs)
        achieved = bytes_env * n / (step_ms * 1e-3) / 1e9
        stream_achieved = bytes_env * n / (gpu_ms / args.steps * 1e-3) / 1e9
        roof = {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_note": traffic_note,
            "bytes_per_env": bytes_env,
            "kernel": f"dd::step_kernel<{'float' if args.precision == 'f32' else 'double'}, 0, true, 0>",
            "us_per_launch": round(step_ms * 1e3, 4),
            "timing": ("GPU wall-clock stamps (dd_stamp: one-lane kernels, s_memrealtime) captured inside the timed "
                       "hipGraphs, at the head of the first and the tail of the last: (their span - the span of a "
                       "graph of the two stamps alone) / K, the K step kernels' own time (the host's graph "
                       "submission excluded; max over ranks)"),
            "span_us": round(span_ms * 1e3, 2),
            "marker_overhead_us": round(marker_ms * 1e3, 2),
            "stream_events": {"us_per_launch": round(gpu_ms / args.steps * 1e3, 4),
                              "frac": round(stream_achieved / HBM_PEAK_GBS, 4),
                              "note": "events on the stream around the graph launches (includes the submission "
                                      "gap before the first kernel)"},
        }
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": pg_world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall * 1e3 / args.steps, 6),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: Philox4x32 random spawns, uniform random 3-bit actions from a device-resident ring",
            "config": {
                "workload": ("config3/config4: 262144 drones per GPU, randomised spawn + auto-reset; "
                             "N GPUs = N x 262144 (config 4 at N=8)" if n == 262_144 else
                             f"{n} drones per GPU, randomised spawn + auto-reset"),
                "envs_per_gpu": n,
                "global_envs": n * pg_world,
                "storage": args.precision,
                "compute": "f64 (reference arithmetic, rounded once on store)",
                "obs": "[N,15] f32 every step" if write_obs else "off",
                "actions": "u8 bitmask [N]",
                "launch": f"hipGraph of {G} steps" if G > 0 else "eager",
                "parallelism": f"env-shard x{pg_world} (no collective on the step path)",
                "world_size_source": ("torch.distributed.get_world_size()" if use_pg else "single process"),
                "launch_form": ("bench.py --gpus N launcher -> torch.distributed.run" if os.environ.get("DD_BENCH_LAUNCHER")
                                else "torch.distributed.run" if "RANK" in os.environ else "plain"),
            },
            "roofline": roof,
            "cpu_baseline": cpu,
            "hbm_point": hbm,
            "rollout_point": c5,
            "step_loop_point": c5a,
            "config2_point": c2,
            "gather_point": gp,
            "gae_point": g5,
            "notebook_reward_point": nb,
            "reinforce_reward_point": rf,
            "f64_point": f64p,
            "ping_pong_point": ppp,
            "policy_point": pp,
            "policy_rollout_point": pr,
            "policy_point_f16x3": pp16,
            "policy_rollout_point_f16x3": pr16,
            "policy_fused_point": pf,
            "policy_fused_point_f16x3": pf16,
            "socket_point": sp,
            "render_point": rp,
            "gpu_ms_per_step": round(step_ms, 6),
            "stream_ms_per_step": round(gpu_ms / args.steps, 6),
            "device": torch.cuda.get_device_name(dev),
            "build_info": abi.lib().dd_build_info().decode(),
        }
        print(json.dumps(out), flush=True)
    if use_pg:
        dist.destroy_process_group()


def pmc_traffic(n: int, precision: str, obs: bool):
    """HBM bytes per launch of the step kernel from the committed rocprofv3 PMC
    summary (profiles/pmc_traffic.json, tools/pmc_summary.py), or None.  A row
    counts only if it was measured on this very build: its build_info (ABI
    version + step-kernel ISA hash) must equal the loaded library's."""
    return pmc_traffic_row(n, precision, obs)[0]


def pmc_traffic_row(n: int, precision: str, obs: bool, path: str | None = None, kernel: str = "step_kernel",
                    frames: int | None = None):
    """(bytes or None, note) — the note says why a row was not taken.  kernel:
    the row's kernel family (rows without a "kernel" key are step_kernel
    rows); frames: the rollout rows' frames per launch."""
    from delivery_drone_amd import abi
    path = path or os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            rows = json.load(f)
    except (OSError, ValueError):
        return None, "no profiles/pmc_traffic.json"
    have = abi.lib().dd_build_info().decode()
    mine = dict(kv.split("=", 1) for kv in have.split(";"))
    for r in rows.get("rows", []):
        if (r.get("envs") == n and r.get("precision") == precision and r.get("obs") == obs
                and r.get("kernel", "step_kernel") == kernel and r.get("frames") == frames):
            got = r.get("build_info")
            if not got:
                return None, "PMC row has no build_info (measured on an older build)"
            theirs = dict(kv.split("=", 1) for kv in got.split(";"))
            # the kernel's own ISA hash when both builds carry it (tools/build_info.py), else the whole unit's
            key = f"{kernel}_isa" if f"{kernel}_isa" in theirs and f"{kernel}_isa" in mine else "step_isa"
            if theirs.get(key) != mine.get(key):
                return None, f"PMC row measured on {key} of '{got}', this library is '{have}'"
            return r.get("hbm_bytes_per_launch"), (f"PMC FETCH_SIZE/WRITE_SIZE passes of the {kernel}; its ISA "
                                                   f"({key}={mine.get(key)}) matches this library's")
    return None, f"no PMC row for {kernel} envs={n} precision={precision} obs={obs} frames={frames}"


if __name__ == "__main__":
    main()
