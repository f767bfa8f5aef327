"""GPU: batches past one launch chunk.

The kernels address a lane array as SGPR base + 32-bit byte offset, so the
host splits every launch into chunks of 2^28 lanes (kChunk in
csrc/drone_step.hip: lane x 8 B stays below 2^31 for f64 storage) and offsets
the SoA, action, output and observation pointers per chunk.  Nothing smaller
than 2^28 + 1 lanes runs a second chunk, so these tests build such a batch
(~32-70 GB of device memory; MI355X has 288 GB) and check, against the
oracle, windows of lanes on both sides of the chunk boundary and at the end of
the batch: reset spawns (keyed by global env id), 60 dd_step frames (the
last collecting done_idx), and a two-frame dd_rollout with observations
(frame stride N x 60 B = 16 GB, so the rollout's 64-bit frame offsets are
exercised too).  Tolerances as in test_gpu_parity.py's oracle comparison:
flags, status, steps and episode exact, floats within 1 float32 ulp.
"""
import numpy as np
import pytest
import torch

import golden_data as gd
from delivery_drone_amd import EnvConfig, VecDroneEnv
from oracle import oracle as ora

pytestmark = pytest.mark.gpu

CHUNK = 1 << 28
N = CHUNK + 4133  # ragged: the second chunk is 17 blocks, the last one partial
WINDOWS = [(0, 2000), (CHUNK - 6000, CHUNK + 4133)]  # the start, and across the boundary to the end


def host(t):
    return t.detach().cpu().numpy()


def window_state(env, lo, hi):
    return {f: host(getattr(env, f)[lo:hi]) for f in gd.FLOAT_FIELDS + ("status", "steps", "episode")}


def check_frame(obs, reward, done, oobs, oreward, odone):
    np.testing.assert_array_equal(done, odone)
    assert gd.f32_close(obs, oobs, 1.0).all()
    assert gd.f32_close(reward, oreward, 1.0).all()


def check_state(env, o, lo, hi):
    got = window_state(env, lo, hi)
    for f in ("status", "steps", "episode"):
        np.testing.assert_array_equal(got[f], getattr(o, f), err_msg=f)
    for f in gd.FLOAT_FIELDS:
        assert gd.f32_close(got[f], getattr(o, f), 1.0).all(), f


@pytest.fixture(scope="module")
def big_env(gpu_device):
    if torch.cuda.get_device_properties(gpu_device).total_memory < 120 * 2**30:
        pytest.skip("needs a large-memory GPU")
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=21)
    env = VecDroneEnv(N, device=gpu_device, config=cfg)
    yield env, cfg
    del env
    torch.cuda.empty_cache()


def test_reset_and_steps_across_chunks(big_env, gpu_device):
    env, cfg = big_env
    obs = env.reset()
    torch.cuda.synchronize()
    oracles = {}
    for lo, hi in WINDOWS:
        o = ora.OracleEnv(hi - lo, precision="f32", config=cfg, env_id_base=lo)
        oobs, _ = o.reset()
        np.testing.assert_array_equal(host(obs[lo:hi]), oobs)  # spawns keyed by the global id
        oracles[(lo, hi)] = o
    g = torch.Generator(device=gpu_device).manual_seed(3)
    frames = 60  # long enough for episodes to end (none does in a spawn's first frames)
    for t in range(frames):
        a = torch.randint(0, 8, (N,), device=gpu_device, generator=g, dtype=torch.uint8)
        obs, reward, done, info = env.step(a, collect_done_idx=(t == frames - 1))
        torch.cuda.synchronize()
        for (lo, hi), o in oracles.items():
            oobs, oreward, odone, _ = o.step(host(a[lo:hi]))
            check_frame(host(obs[lo:hi]), host(reward[lo:hi]), host(done[lo:hi]), oobs, oreward, odone)
            check_state(env, o, lo, hi)
    # the last frame's done_idx: exactly the lanes whose episode ended, global indices
    idx = np.sort(host(info["done_idx"]))
    want = np.flatnonzero(host(done))
    np.testing.assert_array_equal(idx, want)
    assert (idx >= CHUNK).any() and (idx < CHUNK).any()


def test_rollout_across_chunks(big_env, gpu_device):
    env, cfg = big_env
    env.reset()
    torch.cuda.synchronize()
    starts = {w: window_state(env, *w) for w in WINDOWS}
    g = torch.Generator(device=gpu_device).manual_seed(4)
    acts = torch.randint(0, 8, (2, N), device=gpu_device, generator=g, dtype=torch.uint8)
    obs, reward, done = env.rollout(acts)
    torch.cuda.synchronize()
    assert obs.shape == (2, N, 15)
    for (lo, hi), st in starts.items():
        o = ora.OracleEnv(hi - lo, precision="f32", config=cfg, env_id_base=lo)
        o.load_state_dict(st)
        for f in range(2):
            oobs, oreward, odone, _ = o.step(host(acts[f, lo:hi]))
            check_frame(host(obs[f, lo:hi]), host(reward[f, lo:hi]), host(done[f, lo:hi]), oobs, oreward, odone)
        check_state(env, o, lo, hi)
    del obs, reward, done, acts
    torch.cuda.empty_cache()
