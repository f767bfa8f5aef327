"""GPU: BASELINE.json's configurations at their own sizes, through the product
path (VecDroneEnv -> the C ABI -> the HIP kernels), against the C oracle.

* config 1 (1 drone, 1000 frames, fixed spawn): test_gpu_parity.py
  test_config1_trajectory, against the reference's own 1000-frame fixture;
* config 2 (4,096 drones, fixed spawn, f32): here, 256 frames of Philox
  actions, frame by frame, and the same frames as one dd_rollout launch;
* config 3 (262,144 drones, randomised spawn + auto-reset): here, a window
  over 100 frames and then one frame of the whole batch;
* config 4 (2,097,152 drones as 8 shards of 262,144, global env id =
  rank * 262,144 + i; the reference's "parallel games",
  delivery_drone/socket_server.py:113-124): here, on one GPU, the 8 shards
  bit-equal to one 2,097,152-lane batch over 50 frames, a window of every
  shard against the oracle;
* config 5 (65,536 x 256 rollout): test_gpu_rollout.py
  test_config5_shape_against_oracle.

Tolerances: flags, steps and episodes exact; f32 state,
observations and rewards within 1 float32 ulp of the oracle (the frame is
double arithmetic rounded once; device sin/cos and squares may differ from
glibc's by 1 double ulp, which almost never survives the rounding).
"""
import numpy as np
import pytest
import torch

import golden_data as gd
from delivery_drone_amd import EnvConfig, VecDroneEnv
from oracle import oracle as ora

pytestmark = pytest.mark.gpu

STATE = gd.FLOAT_FIELDS + ("status", "steps", "episode")


def host(t):
    return t.detach().cpu().numpy()


def snapshot(env, lo, m):
    return {f: host(getattr(env, f)[lo:lo + m]) for f in STATE}


def assert_frame(obs, reward, done, oobs, oreward, odone, what):
    np.testing.assert_array_equal(done, odone, err_msg=f"{what}: done")
    ok = gd.f32_close(obs, oobs, 1.0)
    assert ok.all(), (what, "obs", np.argwhere(~ok)[:5])
    ok = gd.f32_close(reward, oreward, 1.0)
    assert ok.all(), (what, "reward", np.flatnonzero(~ok)[:5])


def assert_state(env, o, lo, m, what):
    for f in STATE:
        g, r = host(getattr(env, f)[lo:lo + m]), getattr(o, f)
        if f in gd.FLOAT_FIELDS:
            assert gd.f32_close(g, r, 1.0).all(), (what, f)
        else:
            np.testing.assert_array_equal(g, r, err_msg=f"{what}: {f}")


def test_config2_fixed_spawn_4096_f32(gpu_device):
    """Config 2: 4,096 drones, fixed spawn (drone 400,100; pad 400,500), f32
    storage, auto-reset, Philox(seed 0) uniform 3-bit actions per (env, step)
    (include/dronestep.h DD_ACT_PHILOX), 256 frames."""
    n, frames = 4096, 256
    cfg = EnvConfig(randomize_drone=False, randomize_platform=False, auto_reset=True, seed=0)
    env = VecDroneEnv(n, device=gpu_device, config=cfg, precision="f32")
    roll = VecDroneEnv(n, device=gpu_device, config=cfg, precision="f32")
    o = ora.OracleEnv(n, precision="f32", config=cfg)
    obs0 = env.reset()
    roll.reset()
    oobs0, _ = o.reset()
    np.testing.assert_array_equal(host(obs0), oobs0)
    acts = gd.philox_actions_np(0, 0, n, 0, frames)
    acts_d = torch.as_tensor(acts, device=gpu_device)
    r_obs, r_rew, r_done = roll.rollout(frames=frames, action_seed=0, action_step=0)  # the same stream in-kernel
    ends = 0
    for t in range(frames):
        obs, reward, done, _ = env.step(acts_d[t])
        oobs, oreward, odone, _ = o.step(acts[t])
        assert_frame(host(obs), host(reward), host(done), oobs, oreward, odone, f"frame {t}")
        assert torch.equal(r_obs[t], obs) and torch.equal(r_rew[t], reward) and torch.equal(r_done[t], done), t
        ends += int(odone.sum())
    assert_state(env, o, 0, n, "final")
    for f in STATE:
        assert torch.equal(getattr(roll, f), getattr(env, f)), f
    assert ends > 1000 and int(o.episode.max()) > 2  # episodes ended and re-spawned at the fixed spawn


def test_config3_random_spawn_262144(gpu_device):
    """Config 3: 262,144 drones, randomised spawn + auto-reset, seed 0, uniform
    random actions: a 16,384-lane window frame by frame over 100 frames, then
    one frame of the whole batch against the oracle."""
    n, frames, m = 262_144, 100, 16_384
    lo = n - m - 1000  # a window away from the start of the batch
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=0)
    env = VecDroneEnv(n, device=gpu_device, config=cfg)
    env.reset()
    o = ora.OracleEnv(m, precision="f32", config=cfg, env_id_base=lo)
    o.load_state_dict(snapshot(env, lo, m))
    g = torch.Generator(device=gpu_device).manual_seed(0)
    for t in range(frames):
        a = torch.randint(0, 8, (n,), device=gpu_device, generator=g, dtype=torch.uint8)
        obs, reward, done, _ = env.step(a)
        oobs, oreward, odone, _ = o.step(host(a[lo:lo + m]))
        assert_frame(host(obs[lo:lo + m]), host(reward[lo:lo + m]), host(done[lo:lo + m]), oobs, oreward, odone,
                     f"frame {t}")
    assert_state(env, o, lo, m, "window")
    assert int(o.episode.max()) > 1
    full = ora.OracleEnv(n, precision="f32", config=cfg)
    full.load_state_dict(snapshot(env, 0, n))
    a = torch.randint(0, 8, (n,), device=gpu_device, generator=g, dtype=torch.uint8)
    obs, reward, done, _ = env.step(a)
    oobs, oreward, odone, _ = full.step(host(a))
    assert_frame(host(obs), host(reward), host(done), oobs, oreward, odone, "whole batch")
    assert_state(env, full, 0, n, "whole batch")


def test_config4_eight_shards_of_262144(gpu_device):
    """Config 4 on one GPU: 8 VecDroneEnv shards of 262,144 lanes with
    env_id_base = r * 262,144 (bench.py's N=8 layout) step bit for bit as one
    2,097,152-lane batch for 50 frames; a 1,024-lane window of every shard
    (each at a different offset) matches the oracle frame by frame."""
    shard, ranks, frames, m = 262_144, 8, 50, 1024
    n = shard * ranks
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=0)
    full = VecDroneEnv(n, device=gpu_device, config=cfg)
    parts = [VecDroneEnv(shard, device=gpu_device, config=cfg, env_id_base=r * shard) for r in range(ranks)]
    full.reset()
    for p in parts:
        p.reset()
    for f in STATE:
        assert torch.equal(getattr(full, f), torch.cat([getattr(p, f) for p in parts])), f
    offs = [(r * 37_813) % (shard - m) for r in range(ranks)]
    oracles = []
    for r, p in enumerate(parts):
        o = ora.OracleEnv(m, precision="f32", config=cfg, env_id_base=r * shard + offs[r])
        o.load_state_dict(snapshot(p, offs[r], m))
        oracles.append(o)
    g = torch.Generator(device=gpu_device).manual_seed(4)
    for t in range(frames):
        a = torch.randint(0, 8, (n,), device=gpu_device, generator=g, dtype=torch.uint8)
        obs, reward, done, _ = full.step(a)
        for r, p in enumerate(parts):
            sl = slice(r * shard, (r + 1) * shard)
            po, pr, pd, _ = p.step(a[sl])
            assert torch.equal(po, obs[sl]) and torch.equal(pr, reward[sl]) and torch.equal(pd, done[sl]), (t, r)
            w = slice(offs[r], offs[r] + m)
            oo, orr, od, _ = oracles[r].step(host(a[sl][w]))
            assert_frame(host(po[w]), host(pr[w]), host(pd[w]), oo, orr, od, f"frame {t} shard {r}")
    for f in STATE:
        assert torch.equal(getattr(full, f), torch.cat([getattr(p, f) for p in parts])), f
    for r, p in enumerate(parts):
        assert_state(p, oracles[r], offs[r], m, f"shard {r}")
    assert int(full.episode.max()) > 1
