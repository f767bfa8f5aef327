"""GPU: dd_rollout (K frames in one launch) equals K dd_step calls, bit for bit,
and its in-kernel Philox policy equals the documented stream."""
import numpy as np
import pytest
import torch

import golden_data as gd
from delivery_drone_amd import EnvConfig, VecDroneEnv, abi
from oracle import oracle as ora

pytestmark = pytest.mark.gpu


def twins(n, dev, precision="f32", **cfg):
    c = EnvConfig(**cfg)
    a = VecDroneEnv(n, device=dev, config=c, precision=precision)
    b = VecDroneEnv(n, device=dev, config=c, precision=precision)
    a.reset()
    b.reset()
    return a, b


def assert_same_state(a, b):
    for f in gd.FLOAT_FIELDS + ("status", "steps", "episode"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f


@pytest.mark.parametrize("precision", ["f32", "f64"])
@pytest.mark.parametrize("fmt", ["bitmask", "f32x3", "u8x3"])
@pytest.mark.parametrize("n", [1037, 4100])
def test_rollout_equals_step_loop(precision, fmt, n, gpu_device):
    # 1037: no frame row 16-byte aligned past frame 0 (per-frame LDS flush);
    # 4100: full waves take the held double-buffered path, the last 4 rows not
    k = 60
    roll, loop = twins(n, gpu_device, precision, randomize_drone=True, auto_reset=True, seed=3)
    g = torch.Generator(device=gpu_device).manual_seed(2)
    bits = torch.randint(0, 8, (k, n), device=gpu_device, generator=g, dtype=torch.uint8)
    if fmt == "f32x3":
        acts = torch.stack([(bits >> j) & 1 for j in range(3)], dim=2).float()
    elif fmt == "u8x3":
        acts = torch.stack([(bits >> j) & 1 for j in range(3)], dim=2).to(torch.uint8)
    else:
        acts = bits
    obs, reward, done = roll.rollout(acts)
    for t in range(k):
        o, r, d, _ = loop.step(acts[t])
        assert torch.equal(obs[t], o), t
        assert torch.equal(reward[t], r), t
        assert torch.equal(done[t], d), t
    assert_same_state(roll, loop)
    assert int(roll.episode.max()) > 1  # auto-resets happened inside the rollout


def test_rollout_sticky_done_and_outputs_into_buffers(gpu_device):
    n, k = 513, 40
    roll, loop = twins(n, gpu_device, randomize_drone=True, seed=9)
    acts = torch.randint(0, 8, (k, n), device=gpu_device, dtype=torch.uint8)
    buf = torch.zeros(k + 1, n, 15, device=gpu_device)
    rew = torch.zeros(k, n, device=gpu_device)
    dn = torch.zeros(k, n, dtype=torch.bool, device=gpu_device)
    buf[0] = roll.get_state()
    obs, reward, done = roll.rollout(acts, obs_out=buf[1:], reward_out=rew, done_out=dn)
    assert obs.data_ptr() == buf[1].data_ptr() and reward.data_ptr() == rew.data_ptr()
    for t in range(k):
        o, r, d, _ = loop.step(acts[t])
        assert torch.equal(buf[t + 1], o) and torch.equal(rew[t], r) and torch.equal(dn[t], d)
    assert_same_state(roll, loop)
    assert done[-1].any()  # sticky done lanes stay done


def test_rollout_without_obs_and_zero_frames(gpu_device):
    roll, loop = twins(300, gpu_device, randomize_drone=True, auto_reset=True, seed=4)
    acts = torch.randint(0, 8, (25, 300), device=gpu_device, dtype=torch.uint8)
    obs, reward, done = roll.rollout(acts, write_obs=False)
    assert obs is None
    for t in range(25):
        _, r, d, _ = loop.step(acts[t], write_obs=False)
    assert torch.equal(reward[-1], r) and torch.equal(done[-1], d)
    assert_same_state(roll, loop)
    o, r, d = roll.rollout(torch.zeros(0, 300, dtype=torch.uint8, device=gpu_device))
    assert o.shape == (0, 300, 15)
    assert_same_state(roll, loop)


def philox_actions(seed, env0, n, step0, k):
    """include/dronestep.h DD_ACT_PHILOX: step s's bitmask is nibble s & 31 of
    the Philox4x32-10 block (key seed; ctr env, s >> 5), low 3 bits."""
    key = [seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF]
    out = np.zeros((k, n), dtype=np.uint8)
    for t in range(k):
        s = step0 + t
        b = s >> 5
        for i in range(n):
            e = env0 + i
            ctr = [e & 0xFFFFFFFF, e >> 32, b & 0xFFFFFFFF, (b >> 32) ^ 0xA5A5A5A5]
            word = ora.philox4x32_10(ctr, key)[(s >> 3) & 3]
            out[t, i] = (word >> (4 * (s & 7))) & 7
    return out


def test_rollout_philox_policy(gpu_device):
    n, k, env0 = 96, 12, 1000
    c = EnvConfig(randomize_drone=True, auto_reset=True, seed=5)
    roll = VecDroneEnv(n, device=gpu_device, config=c, env_id_base=env0)
    loop = VecDroneEnv(n, device=gpu_device, config=c, env_id_base=env0)
    roll.reset()
    loop.reset()
    obs, reward, done = roll.rollout(frames=k, action_seed=77, action_step=58)  # steps 58-69: two blocks
    acts = torch.as_tensor(philox_actions(77, env0, n, 58, k), device=gpu_device)
    for t in range(k):
        o, r, d, _ = loop.step(acts[t])
        assert torch.equal(obs[t], o) and torch.equal(reward[t], r), t
    assert_same_state(roll, loop)
    assert len({int(a) for a in acts.flatten()}) == 8  # every bitmask drawn


def test_rollout_philox_actions_do_not_depend_on_launch_split(gpu_device):
    # 70 frames from step 5 (blocks of 32 steps: 0-31, 32-63, 64-95) as one launch
    # and as launches of 9, 1, 27, 33 frames: the same actions, the same rollout
    n, k = 200, 70
    c = EnvConfig(randomize_drone=True, auto_reset=True, seed=9)
    one = VecDroneEnv(n, device=gpu_device, config=c)
    split = VecDroneEnv(n, device=gpu_device, config=c)
    one.reset()
    split.reset()
    obs, reward, done = one.rollout(frames=k, action_seed=3, action_step=5)
    parts, t0 = [], 0
    for m in (9, 1, 27, 33):
        parts.append(split.rollout(frames=m, action_seed=3, action_step=5 + t0))
        t0 += m
    assert torch.equal(obs, torch.cat([q[0] for q in parts]))
    assert torch.equal(reward, torch.cat([q[1] for q in parts]))
    assert torch.equal(done, torch.cat([q[2] for q in parts]))
    assert_same_state(one, split)


def test_rollout_philox_sharding_invariant(gpu_device):
    c = EnvConfig(randomize_drone=True, auto_reset=True, seed=6)
    full = VecDroneEnv(2000, device=gpu_device, config=c)
    part = [VecDroneEnv(700, device=gpu_device, config=c),
            VecDroneEnv(1300, device=gpu_device, config=c, env_id_base=700)]
    for e in [full] + part:
        e.reset()
    of, rf, df = full.rollout(frames=150, action_seed=1)
    o0, r0, d0 = part[0].rollout(frames=150, action_seed=1)
    o1, r1, d1 = part[1].rollout(frames=150, action_seed=1)
    assert torch.equal(of, torch.cat([o0, o1], dim=1)) and torch.equal(rf, torch.cat([r0, r1], dim=1))


def test_config5_shape_against_oracle(gpu_device):
    """PPO rollout shape (BASELINE config 5): 65,536 envs x 256 frames in one
    launch; a window of lanes replayed by the oracle with the same actions."""
    n, k = 65_536, 256
    c = EnvConfig(randomize_drone=True, auto_reset=True, seed=8)
    env = VecDroneEnv(n, device=gpu_device, config=c)
    env.reset()
    lo, m = n - 2048, 2048
    o = ora.OracleEnv(m, precision="f32", config=c, env_id_base=lo)
    o.load_state_dict({f: getattr(env, f)[lo:].cpu().numpy() for f in gd.FLOAT_FIELDS + ("status", "steps", "episode")})
    acts = torch.randint(0, 8, (k, n), device=gpu_device, dtype=torch.uint8)
    obs, reward, done = env.rollout(acts)
    a_host = acts[:, lo:].cpu().numpy()
    obs_h, rew_h, done_h = obs[:, lo:].cpu().numpy(), reward[:, lo:].cpu().numpy(), done[:, lo:].cpu().numpy()
    for t in range(k):
        oo, orr, od, _ = o.step(a_host[t])
        np.testing.assert_array_equal(done_h[t], od)
        assert gd.f32_close(obs_h[t], oo, 1.0).all(), t
        assert gd.f32_close(rew_h[t], orr, 1.0).all(), t
    assert torch.isfinite(obs).all()


def test_gae_vs_notebook(gpu_device):
    """dd_gae against compute_gae's own outputs, bit for bit."""
    from delivery_drone_amd import gae
    g = gd.npz("gae.npz")
    dev = gpu_device
    adv, ret = gae(torch.as_tensor(g["rewards"], device=dev), torch.as_tensor(g["values"], device=dev),
                   torch.as_tensor(g["dones"], device=dev), float(g["gamma"]), float(g["lam"]))
    np.testing.assert_array_equal(adv.cpu().numpy(), g["advantages"])
    np.testing.assert_array_equal(ret.cpu().numpy(), g["returns"])
    # T-row values: bootstrap 0 appended, as compute_gae does
    adv0 = gae(torch.as_tensor(g["rewards"], device=dev), torch.as_tensor(g["values"][:-1], device=dev),
               torch.as_tensor(g["dones"], device=dev), returns=False)
    want = ora.gae(g["rewards"], np.concatenate([g["values"][:-1], np.zeros((1, g["values"].shape[1]),
                                                                             np.float32)]), g["dones"])
    np.testing.assert_array_equal(adv0.cpu().numpy(), want)


def test_gae_on_a_rollout_large(gpu_device):
    """Config-5 shaped buffers straight from dd_rollout into dd_gae."""
    from delivery_drone_amd import gae
    n, k = 65_536, 256
    env = VecDroneEnv(n, device=gpu_device, randomize_drone=True, auto_reset=True, seed=2)
    env.reset()
    obs, reward, done = env.rollout(frames=k)
    values = torch.randn(k + 1, n, device=gpu_device)
    adv, ret = gae(reward, values, done)
    lo = n - 512
    want = ora.gae(reward[:, lo:].cpu().numpy(), values[:, lo:].cpu().numpy(), done[:, lo:].cpu().numpy())
    np.testing.assert_array_equal(adv[:, lo:].cpu().numpy(), want)


def test_rollout_large_ragged_equals_step_loop(gpu_device):
    """More lanes than one 2^18-lane wave of blocks, ragged tail."""
    n, k = 262_144 + 1037, 24
    roll, loop = twins(n, gpu_device, "f32", randomize_drone=True, auto_reset=True, seed=13)
    acts = torch.randint(0, 8, (k, n), device=gpu_device, dtype=torch.uint8)
    obs, reward, done = roll.rollout(acts)
    for t in range(k):
        o, r, d, _ = loop.step(acts[t])
        assert torch.equal(obs[t], o) and torch.equal(reward[t], r) and torch.equal(done[t], d), t
    assert_same_state(roll, loop)


@pytest.mark.parametrize("precision", ["f32", "f64"])
@pytest.mark.parametrize("auto", [True, False])
def test_split_rollout_full_chip_equals_step_loop(precision, auto, gpu_device):
    """One block per CU (the split kernel's frame / writer waves: 65,532 lanes,
    the last wave 60 rows), an odd frame count, both done modes."""
    n, k = 65_532, 9
    roll, loop = twins(n, gpu_device, precision, randomize_drone=True, auto_reset=auto, seed=21)
    warm = torch.randint(0, 8, (150, n), device=gpu_device, dtype=torch.uint8)
    roll.rollout(warm)  # mid-episode lanes, some done
    loop.rollout(warm)
    assert_same_state(roll, loop)
    acts = torch.randint(0, 8, (k, n), device=gpu_device, dtype=torch.uint8)
    obs, reward, done = roll.rollout(acts)
    assert roll.last_rollout_kernel == "split"
    for t in range(k):
        o, r, d, _ = loop.step(acts[t])
        assert torch.equal(obs[t], o) and torch.equal(reward[t], r) and torch.equal(done[t], d), t
    assert_same_state(roll, loop)
    roll.check_device_errors()  # no hand-over wait ran out


@pytest.mark.parametrize("precision", ["f32", "f64"])
@pytest.mark.parametrize("n", [777, 4100])
@pytest.mark.parametrize("cfg", [dict(platform_moving=True), dict(wind_enabled=True, wind_x=0.05, wind_y=-0.02),
                                 dict(auto_reset=False), dict(gravity=0.31, auto_reset=True)])
def test_rollout_switches(cfg, n, precision, gpu_device):
    """dd_rollout with the moving platform, wind, sticky done and non-reference
    physics: the kernels without compile-time constants (where ROCm 7.2 once
    miscompiled the f64 observation, tools/scan_isa.py), both obs paths."""
    roll, loop = twins(n, gpu_device, precision, randomize_drone=True, seed=14, **cfg)
    acts = torch.randint(0, 8, (80, n), device=gpu_device, dtype=torch.uint8)
    obs, reward, done = roll.rollout(acts)
    for t in range(80):
        o, r, d, _ = loop.step(acts[t])
        assert torch.equal(obs[t], o) and torch.equal(reward[t], r) and torch.equal(done[t], d), t
    assert_same_state(roll, loop)


@pytest.mark.parametrize("frames", [1, 2, 3])
def test_split_rollout_few_frames_equal_step_loop(frames, gpu_device):
    """The split kernel's hand-over at its edges: one, two and three frames
    (one slot used, both slots, a slot reused), a ragged last block."""
    n = 4100
    roll, loop = twins(n, gpu_device, "f32", randomize_drone=True, auto_reset=True, seed=31)
    warm = torch.randint(0, 8, (40, n), device=gpu_device, dtype=torch.uint8)
    roll.rollout(warm)
    loop.rollout(warm)
    acts = torch.randint(0, 8, (frames, n), device=gpu_device, dtype=torch.uint8)
    obs, reward, done = roll.rollout(acts)
    for t in range(frames):
        o, r, d, _ = loop.step(acts[t])
        assert torch.equal(obs[t], o) and torch.equal(reward[t], r) and torch.equal(done[t], d), t
    assert_same_state(roll, loop)


@pytest.mark.parametrize("precision", ["f32", "f64"])
@pytest.mark.parametrize("n", [777, 65_532])
def test_rollout_short_episodes_equal_step_loop(precision, n, gpu_device):
    """Episodes of a few frames (max_fuel 1.5: out of fuel after one or two
    thrusting frames), so lanes end several episodes between two refills of
    the rollout's drawn-ahead re-spawn blocks (frame.h SpawnAhead, every 32nd
    frame): both the drawn-ahead and the in-frame draw, bit for bit the step
    loop's.  max_fuel 1.5 is not config.py's physics, so this is the single-role
    kernel at both sizes; the split kernel's twin is the next test."""
    k = 37
    roll, loop = twins(n, gpu_device, precision, randomize_drone=True, randomize_platform=True, auto_reset=True,
                       seed=23, max_fuel=1.5)
    acts = torch.randint(0, 8, (k, n), device=gpu_device, dtype=torch.uint8)
    obs, reward, done = roll.rollout(acts)
    for t in range(k):
        o, r, d, _ = loop.step(acts[t])
        assert torch.equal(obs[t], o) and torch.equal(reward[t], r) and torch.equal(done[t], d), t
    assert_same_state(roll, loop)
    assert int(roll.episode.max()) >= 8  # several episodes between two refills on some lanes


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_split_rollout_reference_short_episodes_equal_step_loop(precision, gpu_device):
    """The split kernel (config.py's physics) with lanes that end two episodes
    inside one 32-frame refill interval, so its in-frame re-spawn draw runs
    next to the drawn-ahead one: every lane starts just below the top edge
    climbing (out of bounds on frame 0), and with the main engine on at angle 0
    a re-spawn at y <= ~65 leaves through the top again within ~28 frames."""
    n, k = 65_532, 64
    roll, loop = twins(n, gpu_device, precision, randomize_drone=True, auto_reset=True, seed=41)
    for env in (roll, loop):
        env.y.fill_(-48.0)
        env.vy.fill_(-5.0)
    acts = torch.ones((k, n), device=gpu_device, dtype=torch.uint8)  # main engine only
    obs, reward, done = roll.rollout(acts)
    assert roll.last_rollout_kernel == "split"
    ends_before_refill = done[:31].sum(dim=0)
    for t in range(k):
        o, r, d, _ = loop.step(acts[t])
        assert torch.equal(obs[t], o) and torch.equal(reward[t], r) and torch.equal(done[t], d), t
    assert_same_state(roll, loop)
    assert int((ends_before_refill >= 2).sum()) > 100  # two episodes ended before frame 31 on these lanes
    roll.check_device_errors()


def test_split_rollout_handover_timeout_is_reported(gpu_device):
    """a split-rollout hand-over wait that runs out is not silent.
    kernel="no_wait" caps the waits at zero polls (the frame and writer waves
    then race ahead of each other); dd_device_errors reports DD_ERR_HANDOVER,
    the normal launch does not, and the bits clear once read."""
    n = 65_532
    env = VecDroneEnv(n, device=gpu_device, config=EnvConfig(randomize_drone=True, auto_reset=True, seed=3))
    env.reset()
    env.check_device_errors()
    acts = torch.randint(0, 8, (64, n), device=gpu_device, dtype=torch.uint8)
    env.rollout(acts)
    assert env.last_rollout_kernel == "split"
    env.check_device_errors()
    env.rollout(acts, kernel="no_wait")
    assert env.last_rollout_kernel == "split"
    with pytest.raises(abi.NativeLibraryError, match="DD_ERR_HANDOVER"):
        env.check_device_errors()
    env.check_device_errors()  # read and cleared


def test_device_errors_wait_for_side_streams(gpu_device):
    """dd_device_errors synchronises the device, so a no_wait
    rollout still queued on a non-blocking torch stream (behind a ~20 ms spin
    there) has run and set its bit before check_device_errors() reads it, with
    no synchronize by the caller."""
    n = 65_532
    env = VecDroneEnv(n, device=gpu_device, config=EnvConfig(randomize_drone=True, auto_reset=True, seed=5))
    env.reset()
    env.check_device_errors()
    acts = torch.randint(0, 8, (64, n), device=gpu_device, dtype=torch.uint8)
    torch.cuda.synchronize(gpu_device)
    side = torch.cuda.Stream(gpu_device)
    with torch.cuda.stream(side):
        torch.cuda._sleep(50_000_000)
        env.rollout(acts, kernel="no_wait")
    with pytest.raises(abi.NativeLibraryError, match="DD_ERR_HANDOVER"):
        env.check_device_errors()
    env.check_device_errors()


def test_rollout_kernel_single_equals_split(gpu_device):
    """kernel="single" keeps the single-role kernel where the split one
    applies; both equal the same frames bit for bit."""
    n, k = 65_532, 40
    a, b = twins(n, gpu_device, "f32", randomize_drone=True, auto_reset=True, seed=17)
    acts = torch.randint(0, 8, (k, n), device=gpu_device, dtype=torch.uint8)
    oa, ra, da = a.rollout(acts)
    assert a.last_rollout_kernel == "split"
    ob, rb, db = b.rollout(acts, kernel="single")
    assert b.last_rollout_kernel == "held"
    assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db)
    assert_same_state(a, b)


def test_rollout_launch_groups_past_4gib_of_actions(gpu_device):
    """dd_rollout reads actions by raw buffer loads with 32-bit
    offsets, so rollout_chunks splits a rollout whose action rows span more than
    4 GiB into several launches, passing the state through memory.  f32x3
    actions at 2^22 + 37 lanes (50.3 MB per frame) over 90 frames make two
    launches (85 + 5 frames); the result equals the same frames as 10-frame
    rollouts (each under 4 GiB) bit for bit, the ragged tail included."""
    n, k = (1 << 22) + 37, 90
    roll, loop = twins(n, gpu_device, "f32", randomize_drone=True, auto_reset=True, seed=19)
    g = torch.Generator(device=gpu_device).manual_seed(5)
    bits = torch.randint(0, 8, (k, n), device=gpu_device, generator=g, dtype=torch.uint8)
    acts = torch.empty(k, n, 3, device=gpu_device)
    for j in range(3):
        acts[:, :, j] = ((bits >> j) & 1).float()
    del bits
    assert (k - 1) * n * 12 + n * 12 > 2**32  # the action rows span more than 4 GiB
    _, reward, done = roll.rollout(acts, write_obs=False)
    parts_r, parts_d = [], []
    for g0 in range(0, k, 10):
        _, r, d = loop.rollout(acts[g0:g0 + 10], write_obs=False)
        parts_r.append(r)
        parts_d.append(d)
    assert torch.equal(reward, torch.cat(parts_r)) and torch.equal(done, torch.cat(parts_d))
    assert_same_state(roll, loop)
    assert int(roll.episode.max()) > 1


def test_step_out_buffers_equal_rollout(gpu_device):
    """BASELINE config 5(a): one dd_step per frame writing straight into the
    rollout buffers (step(out=...)) equals one dd_rollout launch."""
    n, k = 4100, 30
    roll, loop = twins(n, gpu_device, randomize_drone=True, auto_reset=True, seed=21)
    acts = torch.randint(0, 8, (k, n), device=gpu_device, dtype=torch.uint8)
    obs, reward, done = roll.rollout(acts)
    ob = torch.full((k, n, 15), float("nan"), device=gpu_device)
    rw = torch.full((k, n), float("nan"), device=gpu_device)
    dn = torch.zeros(k, n, dtype=torch.bool, device=gpu_device)
    for t in range(k):
        o, r, d, _ = loop.step(acts[t], out=(ob[t], rw[t], dn[t]))
        assert o.data_ptr() == ob[t].data_ptr() and r.data_ptr() == rw[t].data_ptr()
    assert torch.equal(ob, obs) and torch.equal(rw, reward) and torch.equal(dn, done)
    assert_same_state(roll, loop)
    with pytest.raises(ValueError):
        loop.step(acts[0], out=(ob[0, :10], rw[0], dn[0]))
