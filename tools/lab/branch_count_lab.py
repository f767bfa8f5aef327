#!/usr/bin/env python
"""Which rare branches the config-5 rollout's waves take, launch by launch
(lab build -DDD_EXP_COUNT: frame.h DD_COUNT sites).  Prints, per 256-frame
dd_rollout launch of 65,536 drones, the share of wave-frames that entered:
0 re-spawn, 1 exact redo, 2 near-pad test, 3 bottom-centre sincos,
4 angle-wrap fallback (site 6 counts every wave-frame)."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "reinforcement-learning-101_amd"))
import torch  # noqa: E402
from delivery_drone_amd import EnvConfig, VecDroneEnv, abi  # noqa: E402

NAMES = ["respawn", "exact_redo", "near_pad", "bottom_sincos", "wrap_fallback"]


def main():
    lib = abi.load(os.path.join(REPO, "reinforcement-learning-101_amd", "delivery_drone_amd", "_native", "lab",
                                "lib_count.so"))
    lib.dd_lab_counts.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    dev = torch.device("cuda", 0)
    n, frames = 65536, 256
    env = VecDroneEnv(n, device=dev, config=EnvConfig(randomize_drone=True, randomize_platform=True,
                                                      auto_reset=True, seed=0), library=lib)
    env.reset()
    acts = torch.randint(0, 8, (frames, n), device=dev, dtype=torch.uint8)
    buf = (ctypes.c_ulonglong * 8)()
    lib.dd_lab_counts(buf, 1)
    for rep in range(20):
        env.rollout(acts)
        torch.cuda.synchronize()
        lib.dd_lab_counts(buf, 1)
        total = max(int(buf[6]), 1)
        row = {"launch": rep, "wave_frames": total, "episodes_max": int(env.episode.max()),
               "done_share": round(float(env.status.bitwise_and(1).float().mean()), 4)}
        row.update({k: round(int(buf[i]) / total, 4) for i, k in enumerate(NAMES)})
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
