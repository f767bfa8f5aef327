"""Loading of the committed reference fixtures (tests/golden/) into SoA form.

The fixtures were produced by tests/golden/make_golden.py from the reference
engine itself; this module only reads them (numpy, allow_pickle=False; JSON).
"""
from __future__ import annotations

import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

ST_DONE, ST_LANDED, ST_CRASHED, ST_PLAT_LEFT = 1, 2, 4, 8
FLOAT_FIELDS = ("x", "y", "vx", "vy", "angle", "omega", "fuel", "px", "py", "total_reward")
DYN_FIELDS = ("x", "y", "vx", "vy", "angle", "omega", "fuel", "px", "py")


def npz(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


def js(name: str):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def state_from_inputs(rec: dict) -> dict:
    """SoA initial state (float64 / uint8 / int32 numpy) of a single-step fixture."""
    st = {f: rec[f"in_{f}"].astype(np.float64) for f in DYN_FIELDS}
    st["total_reward"] = rec["in_total"].astype(np.float64)
    st["status"] = (rec["in_done"].astype(np.uint8) * ST_DONE
                    + (rec["in_direction"] < 0).astype(np.uint8) * ST_PLAT_LEFT).astype(np.uint8)
    st["steps"] = rec["in_steps"].astype(np.int32)
    st["episode"] = np.zeros_like(st["steps"])
    return st


def expected_outputs(rec: dict) -> dict:
    e = {f: rec[f"out_{f}"].astype(np.float64) for f in DYN_FIELDS}
    e["total_reward"] = rec["out_total"].astype(np.float64)
    e["reward"] = rec["out_reward"].astype(np.float64)
    e["done"] = rec["out_done"].astype(bool)
    e["landed"] = rec["out_landed"].astype(bool)
    e["crashed"] = rec["out_crashed"].astype(bool)
    e["plat_left"] = rec["out_direction"] < 0
    e["steps"] = rec["out_steps"].astype(np.int64)
    e["obs"] = rec["out_obs"].astype(np.float64)
    e["info_distance"] = rec["out_info_distance"].astype(np.float64)
    e["info_speed"] = rec["out_info_speed"].astype(np.float64)
    return e


def base_state(**kw) -> dict:
    s = dict(x=400.0, y=100.0, vx=0.0, vy=0.0, angle=0.0, omega=0.0, fuel=1000.0, px=400.0, py=500.0,
             steps=0, total=0.0, done=False, direction=1)
    s.update(kw)
    return s


def edge_case_state(case: dict) -> dict:
    """SoA (one lane) state of an edge_cases.json entry."""
    s = case["state"]
    st = {f: np.array([float(s[f])]) for f in DYN_FIELDS}
    st["total_reward"] = np.array([float(s["total"])])
    st["status"] = np.array([(ST_DONE if s["done"] else 0) | (ST_PLAT_LEFT if s["direction"] < 0 else 0)],
                            dtype=np.uint8)
    st["steps"] = np.array([int(s["steps"])], dtype=np.int32)
    st["episode"] = np.zeros(1, dtype=np.int32)
    return st


def ulp32(a) -> np.ndarray:
    """Spacing of float32 at |a| (as float64)."""
    return np.spacing(np.abs(np.asarray(a, dtype=np.float32))).astype(np.float64)


def f32_close(got, ref, ulps: float = 2.0, atol: float = 0.0) -> np.ndarray:
    """|got - ref| <= ulps * ulp32(ref) + atol, elementwise (ref in double)."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    return np.abs(got - ref) <= ulps * ulp32(ref) + atol


def policy_fixture():
    """policy.npz: obs, the notebook models' outputs, and both state_dicts
    ({"actor": {...}, "critic": {...}}, keys without the 'network.' prefix)."""
    d = npz("policy.npz")
    nets = {tag: {k[len(tag) + len(".network."):]: v for k, v in d.items() if k.startswith(tag + ".network.")}
            for tag in ("actor", "critic")}
    return d, nets


def torch_mlp(sd: dict, device="cpu"):
    """The notebooks' network body (Actor_Critic_PPO.ipynb:376-424) as a plain
    torch fp32 module loaded with `sd`: the floating-point reference the HIP
    kernel is compared with.  Sigmoid is appended for the 3-output actor."""
    import torch
    from torch import nn
    k = sd["9.weight"].shape[0]
    layers = [nn.Linear(15, 128), nn.LayerNorm(128), nn.ReLU(), nn.Linear(128, 128), nn.LayerNorm(128), nn.ReLU(),
              nn.Linear(128, 64), nn.LayerNorm(64), nn.ReLU(), nn.Linear(64, k)]
    if k == 3:
        layers.append(nn.Sigmoid())
    net = nn.Sequential(*layers)
    net.load_state_dict({kk: torch.as_tensor(v) for kk, v in sd.items()})
    return net.to(device).eval()


def philox4x32_10_np(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 (Salmon et al., SC'11) over uint32 numpy arrays: the
    vectorised twin of oracle.philox4x32_10 (tests pin the two together)."""
    m0, m1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
    w0, w1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
    mask = np.uint64(0xFFFFFFFF)
    c = [np.asarray(v, dtype=np.uint32).copy() for v in (c0, c1, c2, c3)]
    k0 = np.asarray(k0, dtype=np.uint32).copy()
    k1 = np.asarray(k1, dtype=np.uint32).copy()
    with np.errstate(over="ignore"):
        for r in range(10):
            p0 = m0 * c[0].astype(np.uint64)
            p1 = m1 * c[2].astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & mask).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & mask).astype(np.uint32)
            c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
            if r < 9:
                k0 = k0 + w0
                k1 = k1 + w1
    return c


def philox_actions_np(seed: int, env0: int, n: int, step0: int, k: int) -> np.ndarray:
    """include/dronestep.h DD_ACT_PHILOX for k steps from step0 and n lanes from
    env id env0: step s's bitmask is nibble s & 31 of the Philox4x32-10 block
    (key seed; counter env, s >> 5, with 0xA5A5A5A5 in the high word), low 3 bits."""
    e = np.arange(env0, env0 + n, dtype=np.uint64)
    out = np.zeros((k, n), dtype=np.uint8)
    key0, key1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    blocks = {}
    for t in range(k):
        s = step0 + t
        b = s >> 5
        if b not in blocks:
            blocks = {b: philox4x32_10_np(e & np.uint64(0xFFFFFFFF), e >> np.uint64(32),
                                          np.full(n, b & 0xFFFFFFFF, np.uint32),
                                          np.full(n, ((b >> 32) ^ 0xA5A5A5A5) & 0xFFFFFFFF, np.uint32),
                                          np.full(n, key0, np.uint32), np.full(n, key1, np.uint32))}
        word = blocks[b][(s >> 3) & 3]
        out[t] = (word >> np.uint32(4 * (s & 7))) & np.uint32(7)
    return out
