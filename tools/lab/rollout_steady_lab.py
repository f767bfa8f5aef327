#!/usr/bin/env python
"""Why later config-5 rollout launches run slower than the first ones
(VERDICT r4 "next" 1): per-launch device times of the 65,536 x 256 rollout
under four schedules, with the shader clock sampled between launches
(tools/micro/clock_probe.hip, one wave, ~20 us):

  burst     back-to-back launches (as bench.py / rocprof time them)
  idle      one launch per 50 ms of host sleep (the chip cools / clocks up)
  restore   back-to-back, the state restored before every launch from the
            first launch's starting state (same trajectory every launch)
  burst+p   burst with a clock probe after every launch
  burst+e   burst with an empty one-wave kernel after every launch
  sync      a host synchronize after every launch (no sleep)
  burstN    N back-to-back launches (e.g. burst200)

A sampler thread reads the GPU's sysfs DPM tables (pp_dpm_sclk / mclk / fclk /
socclk: the active level is starred) every millisecond while a schedule runs,
where they are readable, and reports the levels it saw.

Trajectory-dependent work would make `restore` flat and `burst` slow; a
clock that drops under sustained writes would make `idle` fast and the
probed clock fall with the launch time.  One JSON line per schedule.

    python tools/lab/rollout_steady_lab.py [--launches 40]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "reinforcement-learning-101_amd"))

import torch  # noqa: E402

from delivery_drone_amd import EnvConfig, VecDroneEnv  # noqa: E402

PROBE = os.path.join(REPO, "tools", "micro", "libclock_probe.so")


class DpmSampler:
    """Active DPM level of each readable clock domain, sampled every ~1 ms."""

    def __init__(self):
        import glob
        self.files = {}
        for dom in ("sclk", "mclk", "fclk", "socclk"):
            for f in sorted(glob.glob(f"/sys/class/drm/card*/device/pp_dpm_{dom}")):
                try:
                    open(f).read()
                except OSError:
                    continue
                self.files.setdefault(dom, f)  # the first readable card
        self.seen = {}
        self._stop = None

    def _active(self, f):
        for line in open(f).read().splitlines():
            if line.rstrip().endswith("*"):
                return line.split(":", 1)[-1].strip().rstrip("*").strip()
        return "?"

    def start(self):
        import threading
        self.seen = {d: {} for d in self.files}
        self._stop = threading.Event()

        def loop():
            while not self._stop.is_set():
                for d, f in self.files.items():
                    try:
                        v = self._active(f)
                    except OSError:
                        continue
                    self.seen[d][v] = self.seen[d].get(v, 0) + 1
                time.sleep(0.001)

        self._t = threading.Thread(target=loop, daemon=True)
        self._t.start()

    def stop(self):
        if self._stop is not None:
            self._stop.set()
            self._t.join()
        return self.seen


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=65536)
    p.add_argument("--frames", type=int, default=256)
    p.add_argument("--launches", type=int, default=40)
    p.add_argument("--schedules", default="burst,idle,restore,burst+p")
    p.add_argument("--kernel", default="auto")
    args = p.parse_args()
    dev = torch.device("cuda", 0)
    probe = ctypes.CDLL(PROBE)
    n, frames = args.envs, args.frames
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=0)
    stream = torch.cuda.Stream(dev)
    clk = torch.zeros(args.launches + 1, 3, dtype=torch.int64, device=dev)

    def probe_at(k, iters=20000):
        probe.clock_probe(ctypes.c_void_p(clk[min(k, args.launches)].data_ptr()), iters,
                          ctypes.c_void_p(stream.cuda_stream))

    dpm = DpmSampler()
    print(json.dumps({"dpm_files": dpm.files}), flush=True)
    for sched in args.schedules.split(","):
        launches = int(sched[5:]) if sched.startswith("burst") and sched[5:].isdigit() else args.launches
        env = VecDroneEnv(n, device=dev, config=cfg)
        env.reset()
        torch.manual_seed(1)
        acts = torch.randint(0, 8, (frames, n), device=dev, dtype=torch.uint8)
        obs = torch.empty(frames, n, 15, device=dev)
        rew = torch.empty(frames, n, device=dev)
        done = torch.empty(frames, n, device=dev, dtype=torch.bool)
        start = env.state_dict()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * launches)]
        clk.zero_()
        torch.cuda.synchronize(dev)
        if sched == "idle":
            time.sleep(0.5)
        dpm.start()
        t0 = time.perf_counter()
        with torch.cuda.stream(stream):
            if sched.endswith("+p"):
                probe_at(args.launches)  # the clock before the first launch
            for k in range(launches):
                if sched == "idle":
                    torch.cuda.synchronize(dev)
                    time.sleep(0.05)
                if sched == "restore":
                    env.load_state_dict(start)
                ev[2 * k].record(stream)
                env.rollout(acts, obs_out=obs, reward_out=rew, done_out=done, kernel=args.kernel)
                ev[2 * k + 1].record(stream)
                if sched.endswith("+p"):
                    probe_at(k)
                elif sched.endswith("+e"):
                    probe_at(args.launches, 0)
                elif sched == "sync":
                    torch.cuda.synchronize(dev)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        seen = dpm.stop()
        us = [ev[2 * k].elapsed_time(ev[2 * k + 1]) * 1e3 for k in range(launches)]
        row = {"schedule": sched, "envs": n, "frames": frames, "kernel": env.last_rollout_kernel,
               "us_per_launch": [round(u, 1) for u in us],
               "first5_median": round(statistics.median(us[:5]), 1),
               "last20_median": round(statistics.median(us[-20:]), 1),
               "mean_all": round(statistics.mean(us), 1), "wall_s": round(wall, 4),
               "episodes_started": int(env.episode.sum().item()), "dpm_levels_seen": seen}
        if sched.endswith("+p"):
            c = clk.cpu().tolist()
            ghz = [round(t / r / 10.0, 3) if r else None for t, r, _ in c]  # shader clocks per 10 ns tick
            row["probe_ghz_before_first"] = ghz[args.launches]
            row["probe_ghz_after_launch"] = ghz[:launches]
        env.check_device_errors()
        print(json.dumps(row), flush=True)
        del env, acts, obs, rew, done
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
