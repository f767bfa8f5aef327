"""CPU: the multi-GPU path's host logic — contiguous env-id shards, Philox
keyed by global id (results independent of world size), the gathers of the
observation block and of the whole state to one rank (sharding.gather_obs /
gather_state, the product code tools/multirank_check.py runs on the GPUs) and
bench.py's max-over-ranks timing reduction — rehearsed with the gloo backend
at world_size 2.

The stepping inside each rank is the oracle's here: the product has no CPU
stepping path, and this container has no GPU.  The same
orchestration with VecDroneEnv stepping every shard on the GPU is
tests/test_gpu_multirank.py (two gloo ranks sharing GPU 0, driver-run) and
tests/test_gpu_parity.py::test_sharding_invariance.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as tmp

from delivery_drone_amd import shard_bounds
from delivery_drone_amd.config import EnvConfig
from delivery_drone_amd.sharding import gather_obs, gather_state

TOTAL, FRAMES = 1001, 120


@pytest.mark.parametrize("total,world", [(0, 1), (1, 2), (10, 3), (262_144 * 8, 8), (1001, 2), (7, 8)])
def test_shard_bounds_partition(total, world):
    spans = [shard_bounds(total, r, world) for r in range(world)]
    assert sum(c for _, c in spans) == total
    pos = 0
    for start, count in spans:
        assert start == pos and count >= 0
        pos += count
    counts = [c for _, c in spans]
    assert max(counts) - min(counts) <= 1


def test_shard_bounds_rejects_bad_args():
    with pytest.raises(ValueError):
        shard_bounds(10, 2, 2)
    with pytest.raises(ValueError):
        shard_bounds(-1, 0, 1)


def _actions(frame):
    return np.random.default_rng(1000 + frame).integers(0, 8, TOTAL).astype(np.uint8)


def _cfg():
    return EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=77)


FIELDS = ("x", "y", "vx", "vy", "angle", "omega", "fuel", "px", "py", "total_reward", "status", "steps", "episode")


def _rank_main(rank, world, port, outdir):
    import time
    import bench
    from oracle import oracle as ora
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    start, count = shard_bounds(TOTAL, rank, world)
    env = ora.OracleEnv(count, precision="f32", config=_cfg(), env_id_base=start)
    env.reset()
    t0 = time.perf_counter()
    for t in range(FRAMES):
        obs, reward, done, _ = env.step(_actions(t)[start:start + count])
    wall = bench.reduce_max([time.perf_counter() - t0], "gloo", torch.device("cpu"))[0]
    full = gather_obs(torch.from_numpy(obs), TOTAL, dst=0)
    payload = {"reward": torch.from_numpy(reward.astype(np.float32)), "done": torch.from_numpy(done.astype(np.int32))}
    payload.update({f: torch.from_numpy(getattr(env, f).copy()) for f in FIELDS})
    state = gather_state(payload, TOTAL, dst=0)
    if rank == 0:
        np.savez(os.path.join(outdir, "gathered.npz"), obs=full.numpy(), wall=wall,
                 **{k: v.numpy() for k, v in state.items()})
    else:
        assert full is None and state is None
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_gloo_matches_single_batch(tmp_path):
    from oracle import oracle as ora
    ora.build()
    tmp.spawn(_rank_main, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    g = np.load(tmp_path / "gathered.npz")
    env = ora.OracleEnv(TOTAL, precision="f32", config=_cfg())
    env.reset()
    for t in range(FRAMES):
        obs, reward, done, _ = env.step(_actions(t))
    assert g["obs"].shape == (TOTAL, 15)
    np.testing.assert_array_equal(g["obs"], obs)
    np.testing.assert_array_equal(g["reward"], reward.astype(np.float32))
    np.testing.assert_array_equal(g["done"], done.astype(np.int32))
    for f in FIELDS:  # every SoA field of every shard, in global env-id order
        np.testing.assert_array_equal(g[f], getattr(env, f), err_msg=f)
    assert float(g["wall"]) > 0
    assert env.episode.max() > 1  # episodes ended and re-spawned inside the window


def _edge_main(rank, world, port, outdir):
    """gather_state with an empty shard (total < world) and each rank passing
    its fields in a different dict order."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    total = 2
    start, count = shard_bounds(total, rank, world)
    ids = torch.arange(start, start + count)
    fields = {"a": ids.to(torch.float32), "b": torch.stack([ids, -ids], 1).to(torch.float32),
              "c": ids.to(torch.int32)}
    if rank % 2:  # another insertion order on the odd ranks
        fields = dict(reversed(list(fields.items())))
    state = gather_state(fields, total, dst=0)
    if rank == 0:
        np.savez(os.path.join(outdir, "edge.npz"), **{k: v.numpy() for k, v in state.items()})
    dist.barrier()
    dist.destroy_process_group()


def test_gather_state_empty_shard_and_field_order(tmp_path):
    tmp.spawn(_edge_main, args=(3, _free_port(), str(tmp_path)), nprocs=3, join=True)
    g = np.load(tmp_path / "edge.npz")
    np.testing.assert_array_equal(g["a"], [0.0, 1.0])
    np.testing.assert_array_equal(g["b"], [[0.0, 0.0], [1.0, -1.0]])
    np.testing.assert_array_equal(g["c"], [0, 1])
