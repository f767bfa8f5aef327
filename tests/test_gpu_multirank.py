"""GPU: the product's multi-process path in the driver's GPU tests (BASELINE
config 4's layout, the reference's "parallel games":
delivery_drone/socket_server.py:113-124).

tools/multirank_check.py runs under torch.distributed.run as two gloo ranks
sharing GPU 0: each rank steps its shard (sharding.shard_bounds,
env_id_base) with VecDroneEnv — half the frames as one dd_rollout launch with
in-kernel Philox actions, half as dd_step launches on the shard's slice of
whole-batch actions — then sharding.gather_obs / gather_state bring every
shard's observations, reward, done and SoA state to rank 0, which compares
them bit for bit with the same frames run as ONE batch in a fresh child
process.  RCCL itself needs one GPU per rank (an 8-GPU node, the driver's
scaling run); the orchestration, the keying by global id and the gathers are
the same code.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_two_gloo_ranks_on_gpu0_equal_one_batch(tmp_path, gpu_device):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    total, frames = 2 * 65_536 + 777, 120  # ragged: the shards differ by one drone
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(REPO, "tools", "multirank_check.py"), "--backend", "gloo", "--out", str(tmp_path),
           "--total", str(total), "--frames", str(frames)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=REPO)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    res = json.load(open(tmp_path / "multirank.json"))
    assert res["world"] == 2 and res["backend"] == "gloo" and res["total"] == total
    assert [c for _, c in res["shards"]] == [65_536 + 389, 65_536 + 388]
    assert res["episodes_max"] > 1  # episodes ended and re-spawned inside the window
    assert res["bit_equal"], res["checks"]
    assert set(res["checks"]) >= {"obs", "reward", "done", "x", "status", "episode"}
