"""GPU: bench.py's ping_pong_point alone (VecDroneEnv(ping_pong=True) vs in place, config 3)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "reinforcement-learning-101_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 262_144
print(json.dumps(bench.ping_pong_point(n, 0, torch.device("cuda", 0), rounds=int(os.environ.get("ROUNDS", "5")))))
