"""GPU: the HIP path (through the C ABI) against the reference fixtures and the
oracle, on identical inputs.

Tolerances:
* f64 storage: state / reward / obs within 4 double ulps of the reference
  (|d| <= 4 ulp(ref) + 1e-12 absolute for cancellations near 0); flags exact.
  The kernel does the reference's double arithmetic; differences come only
  from device sin/cos vs glibc (<= 1 ulp) and v*v vs glibc pow(v, 2) (1 ulp
  on ~0.09 % of squares).
* f32 storage: the same double result rounded once to float32, so within
  1 float32 ulp of the reference (2 allowed) and flags exact.
"""
import ctypes
import numpy as np
import pytest
import torch

import golden_data as gd
from delivery_drone_amd import EnvConfig, VecDroneEnv, abi
from oracle import oracle as ora

pytestmark = pytest.mark.gpu


def load(env: VecDroneEnv, st: dict):
    for k, v in st.items():
        t = getattr(env, k)
        t.copy_(torch.as_tensor(np.asarray(v), dtype=t.dtype))


def f64_close(got, ref, ulps=4, atol=1e-12):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    return np.abs(got - ref) <= ulps * np.spacing(np.abs(ref)) + atol


def host(t):
    return t.detach().cpu().numpy()


def step_fixture(rec, precision, device, action_format="bitmask", **cfg):
    n = rec["in_x"].shape[0]
    env = VecDroneEnv(n, precision=precision, device=device, config=EnvConfig(**cfg))
    load(env, gd.state_from_inputs(rec))
    a = torch.as_tensor(rec["in_action"], device=device)
    if action_format == "f32x3":
        a = torch.stack([(a >> k) & 1 for k in range(3)], dim=1).float()
    elif action_format == "u8x3":
        a = torch.stack([(a >> k) & 1 for k in range(3)], dim=1).to(torch.uint8)
    elif action_format == "boolx3":
        a = torch.stack([(a >> k) & 1 for k in range(3)], dim=1).bool()
    obs, reward, done, info = env.step(a)
    torch.cuda.synchronize()
    return env, host(obs), host(reward), host(done), info


def check_vs_reference(env, obs, reward, done, info, e, precision):
    close = (lambda g, r: f64_close(g, r)) if precision == "f64" else (lambda g, r: gd.f32_close(g, r, 2.0))
    np.testing.assert_array_equal(done, e["done"])
    status = host(env.status)
    np.testing.assert_array_equal((status & gd.ST_LANDED) != 0, e["landed"])
    np.testing.assert_array_equal((status & gd.ST_CRASHED) != 0, e["crashed"])
    np.testing.assert_array_equal(host(env.steps), e["steps"])
    for f in gd.DYN_FIELDS + ("total_reward",):
        ok = close(host(getattr(env, f)), e[f])
        assert ok.all(), (f, np.flatnonzero(~ok)[:5])
    assert close(reward, e["reward"]).all()
    ok = gd.f32_close(obs, e["obs"], 2.0)  # obs is float32 in both precisions
    assert ok.all(), np.argwhere(~ok)[:5]
    d, sp = host(info["distance_to_platform"]), host(info["speed"])
    if precision == "f64":
        assert close(d, e["info_distance"]).all() and close(sp, e["info_speed"]).all()
    else:  # _get_info reads the stored (float32-rounded) state: allow its rounding too
        slack_d = 0.5 * (gd.ulp32(e["x"]) + gd.ulp32(e["y"]))
        slack_s = 0.5 * (gd.ulp32(e["vx"]) + gd.ulp32(e["vy"]))
        assert gd.f32_close(d, e["info_distance"], 2.0, slack_d).all()
        assert gd.f32_close(sp, e["info_speed"], 2.0, slack_s).all()


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_single_step_vs_reference(precision, gpu_device):
    rec = gd.npz("single_step.npz")
    env, obs, reward, done, info = step_fixture(rec, precision, gpu_device)
    check_vs_reference(env, obs, reward, done, info, gd.expected_outputs(rec), precision)


@pytest.mark.parametrize("fmt", ["f32x3", "u8x3", "boolx3"])
def test_action_formats_match_bitmask(fmt, gpu_device):
    rec = gd.npz("single_step.npz")
    ref = step_fixture(rec, "f32", gpu_device)
    alt = step_fixture(rec, "f32", gpu_device, action_format=fmt)
    for a, b in zip(ref[1:4], alt[1:4]):
        np.testing.assert_array_equal(a, b)


def test_moving_platform_vs_reference(gpu_device):
    rec = gd.npz("single_step_moving.npz")
    e = gd.expected_outputs(rec)
    env, obs, reward, done, info = step_fixture(rec, "f64", gpu_device, platform_moving=True)
    check_vs_reference(env, obs, reward, done, info, e, "f64")
    np.testing.assert_array_equal((host(env.status) & gd.ST_PLAT_LEFT) != 0, e["plat_left"])


def test_wind_vs_reference(gpu_device):
    rec = gd.npz("single_step_wind.npz")
    env, obs, reward, done, info = step_fixture(rec, "f64", gpu_device, wind_enabled=True,
                                                wind_x=float(rec["in_wind_x"]), wind_y=float(rec["in_wind_y"]))
    check_vs_reference(env, obs, reward, done, info, gd.expected_outputs(rec), "f64")


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_edge_cases_vs_reference(precision, gpu_device):
    for case in gd.js("edge_cases.json"):
        if case["f64_only"] and precision == "f32":
            continue
        env = VecDroneEnv(1, precision=precision, device=gpu_device)
        load(env, gd.edge_case_state(case))
        obs, reward, done, info = env.step(torch.tensor([case["action"]], dtype=torch.uint8, device=gpu_device))
        x = case["expect"]
        st = int(env.status[0].item())
        assert bool(done[0].item()) == x["done"], case["name"]
        assert bool(st & gd.ST_LANDED) == x["landed"] and bool(st & gd.ST_CRASHED) == x["crashed"], case["name"]
        assert int(env.steps[0].item()) == x["steps"], case["name"]
        close = f64_close if precision == "f64" else (lambda g, r: gd.f32_close(g, r, 2.0))
        for f in ("x", "y", "vx", "vy", "angle", "omega", "fuel"):
            assert close(getattr(env, f)[0].item(), x[f]), (case["name"], f)
        assert close(reward[0].item(), x["reward"]), case["name"]
        assert gd.f32_close(host(obs[0]), x["obs"], 2.0).all(), case["name"]


def test_notebook_kats(gpu_device):
    for name, k in gd.js("kat_notebooks.json").items():
        env = VecDroneEnv(1, precision="f64", device=gpu_device)
        load(env, gd.edge_case_state({"state": gd.base_state(**k["start"])}))
        a = torch.tensor([k["action"]], dtype=torch.uint8, device=gpu_device)
        for _ in range(k["frames"]):
            obs, reward, done, info = env.step(a)
        row = dict(zip(("drone_x", "drone_y", "drone_vx", "drone_vy", "drone_angle", "drone_angular_vel",
                        "drone_fuel", "platform_x", "platform_y", "distance_to_platform", "dx_to_platform",
                        "dy_to_platform", "speed"), host(obs[0])))
        got = dict(row, reward=reward[0].item(), total_reward=env.total_reward[0].item(),
                   info_angle=env.angle[0].item(), info_distance=info["distance_to_platform"][0].item(),
                   info_speed=info["speed"][0].item(), steps=int(env.steps[0].item()))
        for key, want in k["expect"].items():
            if key in row:  # obs leaves as float32
                assert gd.f32_close(got[key], want, 1.0), (name, key, got[key], want)
            elif key == "steps":
                assert got[key] == want
            else:
                assert f64_close(got[key], want), (name, key, got[key], want)


@pytest.mark.parametrize("precision", ["f32", "f64"])
@pytest.mark.parametrize("extra", [{}, {"gravity": 0.31, "drag": 0.985, "main_thrust_power": 0.65},
                                   {"platform_moving": True}, {"wind_enabled": True, "wind_x": 0.04, "wind_y": -0.01}],
                         ids=["reference", "custom-physics", "moving", "wind"])
def test_vs_oracle_same_precision(precision, extra, gpu_device):
    """Broad random states: GPU vs the C oracle with the same storage width,
    on the compile-time-constant kernels (reference physics) and the ones that
    take the physics from the call (custom constants, wind, moving pad)."""
    rng = np.random.default_rng(3)
    n = 100_003  # ragged: not a multiple of the 256-lane tile
    rec = gd.npz("single_step.npz")
    idx = rng.integers(0, rec["in_x"].shape[0], n)
    st = {k: v[idx] for k, v in gd.state_from_inputs(rec).items()}
    st["x"] = st["x"] + rng.uniform(-5, 5, n)  # new values (double) around the fixture states
    st["vy"] = st["vy"] + rng.uniform(-0.5, 0.5, n)
    dt = np.float64 if precision == "f64" else np.float32
    st = {k: (v.astype(dt) if v.dtype == np.float64 else v) for k, v in st.items()}
    acts = rng.integers(0, 8, n).astype(np.uint8)
    cfg = EnvConfig(auto_reset=True, randomize_drone=True, seed=9, **extra)
    env = VecDroneEnv(n, precision=precision, device=gpu_device, config=cfg)
    oenv = ora.OracleEnv(n, precision=precision, config=cfg)
    load(env, st)
    oenv.load_state_dict(st)
    for t in range(3):
        obs, reward, done, _ = env.step(torch.as_tensor(acts, device=gpu_device))
        oobs, oreward, odone, _ = oenv.step(acts)
        np.testing.assert_array_equal(host(done), odone)
        np.testing.assert_array_equal(host(env.status), oenv.status)
        np.testing.assert_array_equal(host(env.steps), oenv.steps)
        np.testing.assert_array_equal(host(env.episode), oenv.episode)
        ulps = 1.0
        if precision == "f64":
            for f in gd.FLOAT_FIELDS:
                assert f64_close(host(getattr(env, f)), getattr(oenv, f)).all(), f
        else:
            for f in gd.FLOAT_FIELDS:
                assert gd.f32_close(host(getattr(env, f)), getattr(oenv, f), ulps).all(), f
        assert gd.f32_close(host(obs), oobs, 1.0).all()
        acts = rng.integers(0, 8, n).astype(np.uint8)


def replay(t, precision, device, **cfg):
    T, B = t["actions"].shape
    env = VecDroneEnv(B, precision=precision, device=device, config=EnvConfig(**cfg))

    def set_lane(b, x, y, px, py):
        for f, v in (("x", x), ("y", y), ("px", px), ("py", py)):
            getattr(env, f)[b] = v
        for f in ("vx", "vy", "angle", "omega", "total_reward"):
            getattr(env, f)[b] = 0
        env.fuel[b] = env.config.max_fuel
        env.status[b] = 0
        env.steps[b] = 0

    for b in range(B):
        set_lane(b, *t["spawn0"][b])
    ev = {}
    for row in t["events"]:
        ev.setdefault(int(row[0]), []).append(row[1:])
    worst, flag_mismatch = 0.0, 0
    acts = torch.as_tensor(t["actions"], device=device)
    for i in range(T):
        obs, reward, done, _ = env.step(acts[i])
        worst = max(worst, float(np.max(np.abs(host(obs).astype(np.float64) - t["obs"][i]))))
        flag_mismatch += int((host(done) != t["done"][i]).sum())
        for b, x, y, px, py in ev.get(i, []):
            set_lane(int(b), x, y, px, py)
    return worst, flag_mismatch


@pytest.mark.parametrize("precision", ["f32", "f64"])
@pytest.mark.parametrize("name,cfg", [("traj_random.npz", {}), ("traj_moving.npz", {"platform_moving": True})])
def test_trajectories_vs_reference(name, cfg, precision, gpu_device):
    t = gd.npz(name)
    worst, flag_mismatch = replay(t, precision, gpu_device, **cfg)
    assert flag_mismatch == 0
    # obs leave as float32: 1e-6 covers float32 rounding of values < 8;
    # f32 storage adds the drift of float32 state over ~400 frames
    assert worst < (2e-6 if precision == "f64" else 1e-4), worst


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_config1_trajectory(precision, gpu_device):
    """Config 1 (1000 frames, fixed spawn, reset on done) replayed on the GPU."""
    t = gd.npz("traj_fixed.npz")
    env = VecDroneEnv(1, precision=precision, device=gpu_device, randomize_drone=False,
                      randomize_platform=False)
    env.reset()
    acts = torch.as_tensor(t["actions"], device=gpu_device)
    worst = 0.0
    for i in range(acts.shape[0]):
        obs, reward, done, _ = env.step(acts[i:i + 1])
        worst = max(worst, float(np.max(np.abs(host(obs[0]).astype(np.float64) - t["obs"][i]))))
        assert bool(done[0].item()) == bool(t["done"][i]), i
        if done[0].item():
            env.reset()
            assert gd.f32_close(host(env.obs[0]), t["reset_obs"][i], 1.0).all()
    assert worst < (2e-6 if precision == "f64" else 1e-4), worst


def test_sticky_done_and_needs_reset(gpu_device):
    env = VecDroneEnv(4, device=gpu_device, randomize_platform=False)
    env.reset()
    env.y.fill_(700.0)  # below the world: crash next frame
    a = torch.zeros(4, dtype=torch.uint8, device=gpu_device)
    _, r1, d1, _ = env.step(a)
    assert d1.all() and (r1 < -99).all()
    before = {f: getattr(env, f).clone() for f in ("x", "y", "vx", "vy", "steps", "total_reward")}
    _, r2, d2, info = env.step(a)
    assert d2.all() and (r2 == 0).all() and info["needs_reset"].all()
    for f, v in before.items():
        assert torch.equal(getattr(env, f), v), f


def test_auto_reset_next_step(gpu_device):
    cfg = dict(auto_reset=True, randomize_drone=True, seed=4)
    env = VecDroneEnv(3, device=gpu_device, **cfg)
    env.reset()
    ep0 = env.episode.clone()
    env.y.fill_(700.0)
    a = torch.zeros(3, dtype=torch.uint8, device=gpu_device)
    _, r1, d1, _ = env.step(a)
    assert d1.all()
    obs, r2, d2, _ = env.step(a)
    assert (~d2).all() and (r2 == 0).all()
    assert torch.equal(env.episode, ep0 + 1) and (env.steps == 0).all()
    o = ora.OracleEnv(3, precision="f32", config=EnvConfig(**cfg))
    o.episode[:] = host(ep0)  # the oracle draws the same Philox spawn for (env, episode)
    oobs, _ = o.reset()
    np.testing.assert_array_equal(host(obs), oobs)


def test_reset_matches_oracle_and_ranges(gpu_device):
    facts = gd.js("reset_facts.json")
    n = 200_000
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, seed=11)
    env = VecDroneEnv(n, device=gpu_device, config=cfg, precision="f64")
    obs = env.reset()
    o = ora.OracleEnv(n, precision="f64", config=cfg)
    oobs, _ = o.reset()
    for f in gd.FLOAT_FIELDS:
        np.testing.assert_array_equal(host(getattr(env, f)), getattr(o, f), err_msg=f)
    np.testing.assert_array_equal(host(obs), oobs)
    for f, key in (("x", "drone_x"), ("y", "drone_y"), ("px", "platform_x"), ("py", "platform_y")):
        v = host(getattr(env, f))
        assert [int(v.min()), int(v.max())] == facts[key]
    # determinism and masked reset
    m = torch.zeros(n, dtype=torch.bool, device=gpu_device)
    m[::7] = True
    x_before = env.x.clone()
    env.reset(m)
    assert torch.equal(env.x[~m], x_before[~m])
    assert (env.episode[m] == 2).all() and (env.episode[~m] == 1).all()


def test_sharding_invariance(gpu_device):
    cfg = EnvConfig(randomize_drone=True, auto_reset=True, seed=21)
    full = VecDroneEnv(1000, device=gpu_device, config=cfg)
    parts = [VecDroneEnv(300, device=gpu_device, config=cfg),
             VecDroneEnv(700, device=gpu_device, config=cfg, env_id_base=300)]
    for e in [full] + parts:
        e.reset()
    g = torch.Generator(device=gpu_device).manual_seed(0)
    for _ in range(400):
        a = torch.randint(0, 8, (1000,), device=gpu_device, generator=g, dtype=torch.uint8)
        of, rf, df, _ = full.step(a)
        oa, ra, da, _ = parts[0].step(a[:300])
        ob, rb, db, _ = parts[1].step(a[300:])
        assert torch.equal(of, torch.cat([oa, ob])) and torch.equal(df, torch.cat([da, db]))
    assert int(full.episode.max()) > 1


def test_done_idx_compaction(gpu_device):
    n = 50_000
    env = VecDroneEnv(n, device=gpu_device, randomize_drone=True, seed=2)
    env.reset()
    g = torch.Generator(device=gpu_device).manual_seed(1)
    seen = 0
    for _ in range(200):
        was_done = env.done.clone()
        a = torch.randint(0, 8, (n,), device=gpu_device, generator=g, dtype=torch.uint8)
        _, _, done, info = env.step(a, collect_done_idx=True)
        newly = torch.nonzero(done & ~was_done).flatten().to(torch.int32)
        got = torch.sort(info["done_idx"]).values
        assert torch.equal(got, newly)
        seen += newly.numel()
    assert seen > 1000


def test_active_indices_ordered(gpu_device):
    for n in (1, 255, 256, 257, 70_001):
        env = VecDroneEnv(n, device=gpu_device)
        flags = torch.rand(n, device=gpu_device) < 0.3
        idx = env.active_indices(flags)
        assert torch.equal(idx.long(), torch.nonzero(~flags).flatten())


def test_empty_and_tiny_batches(gpu_device):
    env = VecDroneEnv(0, device=gpu_device)
    obs, reward, done, _ = env.step(torch.zeros(0, dtype=torch.uint8, device=gpu_device))
    assert obs.shape == (0, 15) and env.reset().shape == (0, 15)
    assert env.active_indices().numel() == 0
    env1 = VecDroneEnv(1, device=gpu_device)
    env1.reset()
    env1.step(torch.ones(1, dtype=torch.uint8, device=gpu_device))
    assert int(env1.steps[0]) == 1


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_obs_matches_get_state_and_lane_slices(precision, gpu_device):
    n = 4099
    env = VecDroneEnv(n, device=gpu_device, randomize_drone=True, seed=8, precision=precision)
    env.reset()
    a = torch.randint(0, 8, (n,), device=gpu_device, dtype=torch.uint8)
    obs, _, _, _ = env.step(a)
    step_obs = obs.clone()
    again = env.get_state()
    if precision == "f64":
        assert torch.equal(again, step_obs)
    else:  # step's obs comes from the unrounded frame, get_state from the stored floats
        assert gd.f32_close(host(again), host(step_obs), 2.0, 1e-6).all()
    # stepping a lane range equals stepping those lanes in a full batch
    env2 = VecDroneEnv(n, device=gpu_device, randomize_drone=True, seed=8, precision=precision)
    env2.reset()
    o1, _, _, _ = env2.step(a[:1000], lanes=slice(0, 1000))
    o2, _, _, _ = env2.step(a[1000:], lanes=slice(1000, n))
    assert torch.equal(torch.cat([o1, o2]), step_obs)
    for f in gd.FLOAT_FIELDS:
        assert torch.equal(getattr(env2, f), getattr(env, f)), f


def test_hipgraph_capture_matches_eager(gpu_device):
    n, k = 65_536, 16
    cfg = dict(randomize_drone=True, auto_reset=True, seed=6)
    eager = VecDroneEnv(n, device=gpu_device, **cfg)
    graphed = VecDroneEnv(n, device=gpu_device, **cfg)
    eager.reset()
    graphed.reset()
    acts = torch.randint(0, 8, (k, n), device=gpu_device, dtype=torch.uint8)
    s = torch.cuda.Stream(gpu_device)
    s.wait_stream(torch.cuda.current_stream(gpu_device))
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        for i in range(k):
            graphed.step(acts[i])
    graphed.load_state_dict(eager.state_dict())
    graph.replay()
    for i in range(k):
        eager.step(acts[i])
    torch.cuda.synchronize()
    assert torch.equal(graphed.obs, eager.obs)
    for f in gd.FLOAT_FIELDS + ("status", "steps", "episode"):
        assert torch.equal(getattr(graphed, f), getattr(eager, f)), f


def test_large_batch_properties(gpu_device):
    """BASELINE-scale batch: a sampled slice against the oracle, plus
    size-independent invariants over all lanes."""
    n = 1 << 22
    cfg = EnvConfig(randomize_drone=True, auto_reset=True, seed=13)
    env = VecDroneEnv(n, device=gpu_device, config=cfg)
    env.reset()
    g = torch.Generator(device=gpu_device).manual_seed(5)
    for _ in range(20):
        a = torch.randint(0, 8, (n,), device=gpu_device, generator=g, dtype=torch.uint8)
        obs, reward, done, _ = env.step(a)
    torch.cuda.synchronize()
    assert torch.isfinite(obs).all() and torch.isfinite(reward).all()
    assert (env.fuel >= 0).all() and (env.fuel <= 1000).all()
    assert (env.angle.abs() <= 180).all()
    assert ((reward > -101) & (reward < 100)).all()
    # one more frame on a contiguous window, compared with the oracle
    lo, m = n - 70_000, 70_000
    st = {f: host(getattr(env, f))[lo:] for f in gd.FLOAT_FIELDS + ("status", "steps", "episode")}
    o = ora.OracleEnv(m, precision="f32", config=cfg, env_id_base=lo)
    o.load_state_dict(st)
    a = torch.randint(0, 8, (n,), device=gpu_device, generator=g, dtype=torch.uint8)
    obs, reward, done, _ = env.step(a)
    oobs, oreward, odone, _ = o.step(host(a)[lo:])
    np.testing.assert_array_equal(host(done)[lo:], odone)
    assert gd.f32_close(host(obs)[lo:], oobs, 1.0).all()
    assert gd.f32_close(host(reward)[lo:], oreward, 1.0).all()


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_notebook_reward_vs_reference(precision, gpu_device):
    """the notebooks' calc_reward + max_steps timeout,
    fused into the step, against the notebook's own outputs."""
    rec = gd.npz("shaped_reward.npz")
    n = rec["in_x"].shape[0]
    env = VecDroneEnv(n, precision=precision, device=gpu_device, reward_mode="notebook",
                      max_steps=int(rec["max_steps"]))
    load(env, gd.state_from_inputs(rec))
    hist = np.full((2, n), np.nan)
    slot = (rec["in_steps"].astype(np.int64) + 1) & 1
    hist[slot, np.arange(n)] = rec["in_prev"]
    env.shaped_hist.copy_(torch.as_tensor(hist))
    obs, shaped, sdone, info = env.step(torch.as_tensor(rec["in_action"], device=gpu_device))
    np.testing.assert_array_equal(host(sdone), rec["out_shaped_done"])
    want = rec["out_shaped"]
    got = host(shaped).astype(np.float64)
    if precision == "f64":
        ok = f64_close(got, want, 8, 1e-9)  # |terms| up to ~2e3: 1e-9 covers 1-ulp trig in the inputs
    else:
        ok = gd.f32_close(got, want, 2.0, 1e-6)
    assert ok.all(), np.flatnonzero(~ok)[:5]
    # the engine's own reward is still there, unchanged
    e_env, _, e_reward, e_done, _ = step_fixture(rec, precision, gpu_device)
    assert np.array_equal(host(info["engine_reward"]), e_reward)


def test_notebook_reward_kat_and_history(gpu_device):
    k = gd.js("kat_notebooks.json")["actor_critic_ppo"]
    env = VecDroneEnv(1, precision="f64", device=gpu_device, reward_mode="notebook")
    env.reset()
    load(env, gd.edge_case_state({"state": gd.base_state(**k["start"])}))
    env.shaped_hist.fill_(float("nan"))
    _, shaped, _, _ = env.step(torch.tensor([k["action"]], dtype=torch.uint8, device=gpu_device))
    assert shaped[0].item() == k["shaped_total"]


def test_notebook_mode_matches_oracle_over_episodes(gpu_device):
    """Multi-frame: 2-back history, auto-reset restarts it, 300-step timeout."""
    n, frames = 4099, 700
    cfg = EnvConfig(randomize_drone=True, auto_reset=True, seed=12)
    env = VecDroneEnv(n, device=gpu_device, config=cfg, precision="f64", reward_mode="notebook", max_steps=300)
    env.reset()
    o = ora.OracleEnv(n, precision="f64", config=cfg)
    o.reset()
    hist = np.full((2, n), np.nan)
    hist[0] = host(env.shaped_hist)[0]
    assert np.array_equal(hist[0], host(env.shaped_hist)[0])
    rng = np.random.default_rng(3)
    worst, timeouts = 0.0, 0
    for t in range(frames):
        a = rng.integers(0, 8, n).astype(np.uint8)
        _, shaped, sdone, _ = env.step(torch.as_tensor(a, device=gpu_device))
        *_, oshaped, osdone = o.step_shaped(a, hist, 300)
        np.testing.assert_array_equal(host(sdone), osdone)
        worst = max(worst, float(np.max(np.abs(host(shaped) - oshaped))))
        timeouts += int(((host(env.steps) == 300) & host(sdone)).sum())
    assert worst < 1e-9
    assert timeouts > 0  # some episodes hit the 300-step cap


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_reinforce_reward_vs_reference(precision, gpu_device):
    """REINFORCE's calc_reward (Policy_Gradients.ipynb:162-238) + collect_episodes'
    timeout (:590-593), fused into the step, against the notebook's own
    outputs (tests/golden/reinforce_reward.npz).  Tolerance as the PPO reward's:
    the kernel squares with x*x and takes the device's exp, the notebook glibc's
    pow and exp, so terms may differ by an ulp."""
    rec = gd.npz("reinforce_reward.npz")
    n = rec["in_x"].shape[0]
    env = VecDroneEnv(n, precision=precision, device=gpu_device, reward_mode="reinforce",
                      max_steps=int(rec["max_steps"]))
    load(env, gd.state_from_inputs(rec))
    obs, shaped, sdone, info = env.step(torch.as_tensor(rec["in_action"], device=gpu_device))
    np.testing.assert_array_equal(host(sdone), rec["out_shaped_done"])
    want = rec["out_shaped"]
    got = host(shaped).astype(np.float64)
    if precision == "f64":
        ok = f64_close(got, want, 8, 1e-9)
    else:
        ok = gd.f32_close(got, want, 2.0, 1e-6)
    assert ok.all(), np.flatnonzero(~ok)[:5]
    e_env, _, e_reward, e_done, _ = step_fixture(rec, precision, gpu_device)
    assert np.array_equal(host(info["engine_reward"]), e_reward)


def test_reinforce_mode_matches_oracle_over_episodes(gpu_device):
    """Multi-frame REINFORCE mode: auto-reset, the 300-step timeout, against the
    oracle's restatement of the notebook cell."""
    n, frames = 4099, 700
    cfg = EnvConfig(randomize_drone=True, auto_reset=True, seed=13)
    env = VecDroneEnv(n, device=gpu_device, config=cfg, precision="f64", reward_mode="reinforce", max_steps=300)
    env.reset()
    o = ora.OracleEnv(n, precision="f64", config=cfg)
    o.reset()
    rng = np.random.default_rng(4)
    worst, timeouts, landings = 0.0, 0, 0
    for t in range(frames):
        a = rng.integers(0, 8, n).astype(np.uint8)
        _, shaped, sdone, _ = env.step(torch.as_tensor(a, device=gpu_device))
        *_, oshaped, osdone = o.step_shaped(a, None, 300, mode="reinforce")
        np.testing.assert_array_equal(host(sdone), osdone)
        worst = max(worst, float(np.max(np.abs(host(shaped) - oshaped))))
        timeouts += int(((host(env.steps) == 300) & host(sdone)).sum())
    assert worst < 1e-9
    assert timeouts > 0


@pytest.mark.parametrize("precision", ["f32", "f64"])
@pytest.mark.parametrize("auto", [True, False])
def test_ping_pong_equals_in_place(precision, auto, gpu_device):
    """VecDroneEnv(ping_pong=True) (DDStepIO.state_out: read one copy of the
    per-frame fields, write the other) gives the in-place step's bits: every
    output and every field, sticky-done lanes (which must copy their fields
    across) and re-spawns included, and replayed hipGraphs of an even number
    of steps."""
    n, k = 10_007, 120
    cfg = dict(randomize_drone=True, auto_reset=auto, seed=21)
    a = VecDroneEnv(n, device=gpu_device, precision=precision, **cfg)
    b = VecDroneEnv(n, device=gpu_device, precision=precision, ping_pong=True, **cfg)
    a.reset()
    b.reset()
    g = torch.Generator(device=gpu_device).manual_seed(4)
    acts = torch.randint(0, 8, (k, n), device=gpu_device, dtype=torch.uint8, generator=g)
    for t in range(k):
        oa, ra, da, _ = a.step(acts[t])
        ob, rb, db, _ = b.step(acts[t])
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db), t
    for f in gd.FLOAT_FIELDS + ("status", "steps", "episode"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
    assert (a.status & gd.ST_DONE).any()  # done lanes were stepped (sticky or re-spawned)
    # a graph of an even number of steps replays from the copy it ends on
    s = torch.cuda.Stream(gpu_device)
    s.wait_stream(torch.cuda.current_stream(gpu_device))
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        for t in range(4):
            b.step(acts[t])
    for _ in range(3):
        graph.replay()
        for t in range(4):
            a.step(acts[t])
    torch.cuda.synchronize()
    assert torch.equal(a.obs, b.obs)
    for f in gd.FLOAT_FIELDS + ("status", "steps", "episode"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_contiguous_memory_equals_torch_memory(precision, gpu_device):
    """VecDroneEnv(memory="contiguous") (every field and output carved from
    one dd_device_alloc(DD_MEM_CONTIGUOUS) range at 2 MiB boundaries) steps,
    rolls out and resets to the same bits as the default allocation; the
    range is freed with the env's last tensor."""
    from delivery_drone_amd import abi
    n, k = 70_001, 60
    cfg = dict(randomize_drone=True, auto_reset=True, seed=5)
    a = VecDroneEnv(n, device=gpu_device, precision=precision, **cfg)
    b = VecDroneEnv(n, device=gpu_device, precision=precision, memory="contiguous", **cfg)
    assert b.memory == "contiguous"
    ptrs = sorted(getattr(b, f).data_ptr() for f in gd.FLOAT_FIELDS + ("status", "steps", "episode", "obs", "reward"))
    assert all(p % (2 << 20) == ptrs[0] % (2 << 20) for p in ptrs)  # one range, 2 MiB-aligned offsets
    assert ptrs[-1] - ptrs[0] < 64 * (2 << 20) + 8 * n * 16
    a.reset()
    b.reset()
    g = torch.Generator(device=gpu_device).manual_seed(6)
    acts = torch.randint(0, 8, (k, n), device=gpu_device, dtype=torch.uint8, generator=g)
    for t in range(k):
        oa, ra, da, _ = a.step(acts[t])
        ob, rb, db, _ = b.step(acts[t])
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db), t
    ra = a.rollout(acts[:16], frames=16)
    rb = b.rollout(acts[:16], frames=16)
    for x, y in zip(ra, rb):
        assert torch.equal(x, y)
    for f in gd.FLOAT_FIELDS + ("status", "steps", "episode"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
    assert (b.status & gd.ST_DONE).any() or int(b.episode.max()) > 1
    with pytest.raises(ValueError):
        VecDroneEnv(16, device=gpu_device, memory="pinned")
    # the range goes with the last tensor over it
    free0, _ = torch.cuda.mem_get_info(gpu_device)
    big = VecDroneEnv(1 << 22, device=gpu_device, memory="contiguous")
    free1, _ = torch.cuda.mem_get_info(gpu_device)
    assert free0 - free1 >= (1 << 22) * 60
    del big
    import gc
    gc.collect()
    torch.cuda.synchronize(gpu_device)
    free2, _ = torch.cuda.mem_get_info(gpu_device)
    assert free2 - free1 >= (1 << 22) * 60
    assert abi.DD_MEM_CONTIGUOUS == 1


def test_ping_pong_rejects_aliasing_and_lane_slices(gpu_device):
    from delivery_drone_amd import abi
    env = VecDroneEnv(256, device=gpu_device, ping_pong=True)
    env.reset()
    with pytest.raises(ValueError):
        env.step(torch.zeros(128, dtype=torch.uint8, device=gpu_device), lanes=slice(0, 128))
    io = abi.DDStepIO()
    acts = torch.zeros(256, dtype=torch.uint8, device=gpu_device)
    io.actions, io.reward, io.done = acts.data_ptr(), env.reward.data_ptr(), env._done.data_ptr()
    io.state_out = ctypes.cast(ctypes.pointer(env._state), ctypes.c_void_p)  # out aliases in
    stream = torch.cuda.current_stream(gpu_device).cuda_stream
    assert env._lib.dd_step(ctypes.byref(env._cfg), ctypes.byref(env._state), ctypes.byref(io), 256, stream) != 0
    bad = env._make_state(env._twin)
    bad.px = env._twin["x"].data_ptr()  # a shared field that differs
    io.state_out = ctypes.cast(ctypes.pointer(bad), ctypes.c_void_p)
    assert env._lib.dd_step(ctypes.byref(env._cfg), ctypes.byref(env._state), ctypes.byref(io), 256, stream) != 0


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_obs_rows_bit_exact_on_integer_states(precision, gpu_device):
    """The observation columns are x * RN(1/d) (one multiply) instead of the
    reference's x / d (frame.h observe_values): the double may
    differ by an ulp, the float32 row only when the quotient lies within
    ~1e-16 relative of a float32 rounding boundary.  On the states a spawn
    makes — integer drone and pad positions over and past the spawn ranges,
    at rest, full fuel — the rows equal the oracle's (the reference's
    quotients) bit for bit."""
    xs = np.arange(-60, 861, dtype=np.float64)
    ys = np.arange(-60, 661, dtype=np.float64)
    gx, gy = np.meshgrid(xs, ys, indexing="ij")
    n = gx.size
    rng = np.random.default_rng(9)
    st = {f: np.zeros(n) for f in gd.FLOAT_FIELDS}
    st.update(x=gx.ravel(), y=gy.ravel(), px=rng.integers(50, 751, n).astype(np.float64),
              py=rng.integers(100, 551, n).astype(np.float64), fuel=np.full(n, 1000.0),
              angle=rng.integers(-180, 181, n).astype(np.float64))
    st.update(status=np.zeros(n, np.uint8), steps=np.zeros(n, np.int32), episode=np.ones(n, np.int32))
    env = VecDroneEnv(n, device=gpu_device, precision=precision)
    dt = torch.float64 if precision == "f64" else torch.float32
    env.load_state_dict({f: torch.as_tensor(v, dtype=dt if f in gd.FLOAT_FIELDS else None) for f, v in st.items()})
    obs = host(env.get_state())
    o = ora.OracleEnv(n, precision=precision)
    o.load_state_dict(st)
    oobs, _ = o.get_state()
    np.testing.assert_array_equal(obs, oobs)


def test_long_trajectory_drift_vs_reference_math(gpu_device):
    """What the fast sin / cos (trig.h: at most 1 ulp from glibc, 13 % of
    results 1 ulp off since round 3 dropped the reduction's tail word) and
    v*v for glibc's pow(v, 2) do to a long f64 trajectory: 4,096 lanes x 1,000
    frames, random actions, against the oracle (libm exactly as the
    reference), the largest drift of every field in ulps of max(|value|, 1)
    at the end, with flags, steps and episodes still equal.  The bound asserted
    (256 ulps; measured values are reported in the assertion message and in
    DESIGN.md §3.2) keeps the looser per-step trig tolerance backed by data
    (ADVICE r03)."""
    n, k = 4096, 1000
    cfg = EnvConfig(randomize_drone=True, auto_reset=False, seed=3)
    env = VecDroneEnv(n, device=gpu_device, precision="f64", config=cfg)
    o = ora.OracleEnv(n, precision="f64", config=cfg)
    env.reset()
    o.reset()
    rng = np.random.default_rng(17)
    for t in range(k):
        a = rng.integers(0, 8, n).astype(np.uint8)
        a[rng.random(n) < 0.6] &= 6  # fire the main engine less often: longer episodes
        env.step(torch.as_tensor(a, device=gpu_device))
        o.step(a)
    for f in ("status", "steps", "episode"):
        np.testing.assert_array_equal(host(getattr(env, f)), getattr(o, f), err_msg=f)
    drift = {}
    for f in ("x", "y", "vx", "vy", "angle", "omega", "fuel", "total_reward"):
        g, r = host(getattr(env, f)), getattr(o, f)
        drift[f] = float(np.max(np.abs(g - r) / np.spacing(np.maximum(np.abs(r), 1.0))))
    assert all(v <= 256 for v in drift.values()), drift
    print("max drift (ulps) after", k, "frames:", {f: round(v, 1) for f, v in drift.items()})
