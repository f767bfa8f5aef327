"""GPU: the N > 1 bench is launch-ready without torch.distributed.run
(VERDICT r05 next #2).  `python3 bench.py --gpus N` is its own launcher: it
measures the CPU baseline once, starts N ranks as a child
torch.distributed.run (never an exec) and relays rank 0's one JSON line,
whose n_gpus is the process group's own world size.  On the one-GPU box the
two ranks share GPU 0 over gloo; RCCL with fewer GPUs than ranks fails fast.
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _bench(args, timeout):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=REPO)


def test_plain_launch_two_gloo_ranks(gpu_device):
    r = _bench(["--gpus", "2", "--dist-backend", "gloo", "--steps", "20", "--warmup", "5", "--rollout-point", "0",
                "--hbm-point", "0", "--no-extra-points", "--cpu-baseline", "1"], timeout=110)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_envs"] == 2 * 262_144
    assert out["config"]["world_size_source"] == "torch.distributed.get_world_size()"
    assert out["config"]["launch_form"].startswith("bench.py --gpus N launcher")
    cpu = out["cpu_baseline"]
    assert cpu and cpu["value"] > 0 and cpu["kind"] == "port" and "launcher" in cpu["measured_by"]
    gp = out["gather_point"]
    assert gp and "error" not in gp and gp["rows"] == 2 * 262_144, gp
    assert out["value"] > 0 and out["roofline"]["frac"] > 0


def test_plain_launch_nccl_needs_a_gpu_per_rank(gpu_device):
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("two or more GPUs visible")
    r = _bench(["--gpus", "2", "--dist-backend", "nccl", "--steps", "20", "--warmup", "5", "--cpu-baseline", "0"],
               timeout=60)
    assert r.returncode != 0 and "RCCL needs one GPU per rank" in r.stderr, r.stderr[-2000:]
