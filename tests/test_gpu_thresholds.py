"""GPU: done / landed / crashed flags exactly equal to the oracle's (which is
bit-exact to the reference: libm sin, cos and pow, as numpy and CPython
call them) on states placed within a few ulps of every predicate boundary of
the reward cascade — y' = 550, the out-of-bounds margins, speed' = 3,
|angle'| = 20, the four pad edges of the bottom centre, fuel' = 0
(game_engine.py:218-279, drone.py:130-153; tests/threshold_states.py).

A frame evaluates its predicates on doubles that may differ from the
reference's by an ulp (device sin/cos vs glibc, v*v vs glibc pow(v, 2)); near
a boundary the kernel re-evaluates them the reference's way,
so the flags stay exact.  Rewards: exact for terminal frames (the cascade's
constants); shaping frames within 4 ulps + 1e-16 (their distance uses v*v
off the rare path); state within 4 double ulps (f64 storage) or 1 float32 ulp
(f32 storage), as tests/test_gpu_parity.py bounds them."""
import numpy as np
import pytest
import torch

import golden_data as gd
import threshold_states as ts
from delivery_drone_amd import EnvConfig, VecDroneEnv
from oracle import oracle as ora

pytestmark = pytest.mark.gpu

N = 1 << 20


def host(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_flags_exact_near_every_boundary(precision, gpu_device):
    st, acts, fam, dist = ts.generate(N, precision, seed=11 if precision == "f64" else 12)
    assert np.mean(dist <= 16.5) > 0.99  # the states are where they should be
    cfg = EnvConfig()
    env = VecDroneEnv(N, device=gpu_device, precision=precision, config=cfg)
    dt = torch.float64 if precision == "f64" else torch.float32
    for f in gd.FLOAT_FIELDS:
        getattr(env, f).copy_(torch.as_tensor(st[f], dtype=dt))
    for f in ("status", "steps", "episode"):
        getattr(env, f).copy_(torch.as_tensor(st[f]))
    o = ora.OracleEnv(N, precision=precision, config=cfg)
    o.load_state_dict({f: (st[f].astype(np.float32) if precision == "f32" and f in gd.FLOAT_FIELDS else st[f])
                       for f in st})
    obs, reward, done, _ = env.step(torch.as_tensor(acts, device=gpu_device))
    oobs, oreward, odone, _ = o.step(acts)
    g_status, g_reward = host(env.status), host(reward).astype(np.float64)
    bad = (g_status != o.status) | (host(done) != odone)
    report = {name: int(bad[fam == f].sum()) for f, name in enumerate(ts.FAMILIES)}
    assert not bad.any(), f"flag mismatches per family: {report}"
    landed = (o.status & gd.ST_LANDED) != 0
    crashed = (o.status & gd.ST_CRASHED) != 0
    assert landed.sum() > N // 20 and crashed.sum() > N // 20 and (~(landed | crashed)).sum() > N // 20
    term = odone
    np.testing.assert_array_equal(g_reward[term], oreward[term].astype(np.float64))
    if precision == "f64":
        # a shaping reward's distance may differ by an ulp of ~500 (v*v vs pow),
        # 2e-17 after the / 5000: that, or 4 ulps of the reward (test_gpu_parity's bound)
        ok = np.abs(g_reward - oreward) <= 4 * np.spacing(np.abs(oreward)) + 1e-16
        assert ok.all(), np.flatnonzero(~ok)[:5]
        for f in gd.FLOAT_FIELDS:
            g, r = host(getattr(env, f)), getattr(o, f)
            ok = np.abs(g - r) <= 4 * np.spacing(np.abs(r)) + 1e-12
            assert ok.all(), (f, np.flatnonzero(~ok)[:5])
    else:
        assert gd.f32_close(g_reward, oreward, 1.0).all()
        for f in gd.FLOAT_FIELDS:
            assert gd.f32_close(host(getattr(env, f)), getattr(o, f), 1.0).all(), f
    assert gd.f32_close(host(obs), oobs, 1.0).all()


def test_unscaled_sqrt_bit_equal_to_compiler_sqrt(gpu_device):
    """The frame's square roots (speed, distance: drone.py:139-145,
    physics.py:42-44) skip the compiler's scaling of inputs below 2^-767
    (trig.h sqrt_unscaled; smaller ones take sqrt()).  On the device, every
    integer 0..2^20 and 2^26 doubles with exponents spread from 2^-767 to the
    largest finite give the same bits both ways."""
    from delivery_drone_amd import abi
    lib = abi.lib()
    bad = torch.zeros(1, dtype=torch.int64, device=gpu_device)
    stream = torch.cuda.current_stream(gpu_device).cuda_stream
    rc = lib.dd_selftest_sqrt(12345, 1 << 26, bad.data_ptr(), stream)
    assert rc == 0, abi.lib().dd_error_string(rc)
    torch.cuda.synchronize(gpu_device)
    assert int(bad.item()) == 0
