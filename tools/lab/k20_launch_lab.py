"""Where the driver-shaped line's wall time goes (bench.py --steps 20 --warmup 5).

Runs bench.py (headline only) as child processes, interleaved, under launch
settings that change only how the host submits work, and prints one JSON line
per run with the wall and event times per step.  Lab tool: not part of the
product or of the tests.

    python tools/lab/k20_launch_lab.py [--reps 3] [--steps 20]
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

VARIANTS = {
    "base": ({}, []),
    "dev_kernarg": ({"HIP_FORCE_DEV_KERNARG": "1"}, []),
    "graph10": ({}, ["--graph-steps", "10"]),
    "eager": ({}, ["--graph-steps", "0"]),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    a = ap.parse_args()
    names = a.variants.split(",")
    for rep in range(a.reps):
        for name in names:
            env_add, extra = VARIANTS[name]
            env = dict(os.environ, **env_add)
            cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", str(a.steps), "--warmup",
                   str(a.warmup), "--cpu-baseline", "0", "--hbm-point", "0", "--rollout-point", "0",
                   "--no-extra-points"] + extra
            r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                print(json.dumps({"variant": name, "rep": rep, "rc": r.returncode, "err": r.stderr[-400:]}))
                sys.exit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            print(json.dumps({"variant": name, "rep": rep, "steps": a.steps, "value": d["value"],
                              "wall_us_per_step": round(d["ms_per_step"] * 1e3, 3),
                              "event_us_per_step": round(d["gpu_ms_per_step"] * 1e3, 3),
                              "launch": d["config"]["launch"]}), flush=True)


if __name__ == "__main__":
    main()
