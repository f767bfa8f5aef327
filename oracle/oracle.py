"""TEST INFRASTRUCTURE ONLY — numpy/ctypes front end of the CPU oracle.

``liboracle.so`` (drone_oracle.c, built by oracle/Makefile) restates the
reference's frame in scalar IEEE double; :class:`OracleEnv` holds a batch of
lanes in host numpy arrays with exactly the SoA layout and the semantics of
``VecDroneEnv`` / ``dd_step``, so tests can run both on the same inputs and
compare.  Only tests/, ``__graft_entry__.smoke()`` and bench.py's
cpu_baseline leg use this module; the product never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(_HERE)
sys.path.insert(0, os.path.join(_REPO, "reinforcement-learning-101_amd"))

from delivery_drone_amd import abi  # noqa: E402  (struct layouts of include/dronestep.h)
from delivery_drone_amd.config import EnvConfig  # noqa: E402

LIB_PATH = os.path.join(_HERE, "liboracle.so")
FLOAT_FIELDS = ("x", "y", "vx", "vy", "angle", "omega", "fuel", "px", "py", "total_reward")
_LIB = None
_LOCK = threading.Lock()


def build(force: bool = False) -> str:
    """Compile liboracle.so with gcc (oracle/Makefile)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", _HERE] + (["-B"] if force else []), check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        with _LOCK:
            if _LIB is None:
                build()
                h = ctypes.CDLL(LIB_PATH)
                P = ctypes.c_void_p
                cfgp, stp = ctypes.POINTER(abi.DDConfig), ctypes.POINTER(abi.DDState)
                h.ora_step.argtypes = [cfgp, stp, P, P, P, P, P, ctypes.c_int64]
                h.ora_step_shaped.argtypes = [cfgp, stp, P, P, P, P, P, P, P, P, ctypes.c_int32, ctypes.c_int32,
                                              ctypes.c_int64]
                h.ora_notebook_reward.argtypes = [P, ctypes.c_double]
                h.ora_notebook_reward.restype = ctypes.c_double
                h.ora_reinforce_reward.argtypes = [P]
                h.ora_reinforce_reward.restype = ctypes.c_double
                h.ora_reset.argtypes = [cfgp, stp, P, P, P, ctypes.c_int64]
                h.ora_write_obs.argtypes = [cfgp, stp, P, P, ctypes.c_int64]
                h.ora_get_info.argtypes = [cfgp, stp, P, P, ctypes.c_int64]
                h.ora_probe.argtypes = [cfgp, stp, P, P, ctypes.c_int64]
                h.ora_philox4x32_10.argtypes = [P, P, P]
                h.ora_philox4x32_10.restype = None
                h.ora_philox4x32_7.argtypes = [P, P, P]
                h.ora_philox4x32_7.restype = None
                h.ora_bench.argtypes = [cfgp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64]
                h.ora_gae.argtypes = [P, P, P, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_double, ctypes.c_double]
                h.ora_gae.restype = None
                h.ora_bench.restype = ctypes.c_double
                _LIB = h
    return _LIB


def _p(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def philox4x32_10(ctr, key):
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    k = np.ascontiguousarray(key, dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint32)
    lib().ora_philox4x32_10(_p(c), _p(k), _p(out))
    return out


def philox4x32_7(ctr, key):
    """The spawn stream's generator (drone_oracle.c ora_spawn, frame.h spawn_words)."""
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    k = np.ascontiguousarray(key, dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint32)
    lib().ora_philox4x32_7(_p(c), _p(k), _p(out))
    return out


def bitmask(actions) -> np.ndarray:
    """[N] bitmask or [N, 3] (main, left, right) truthy values -> uint8 bitmask."""
    a = np.asarray(actions)
    if a.ndim == 2:
        a = ((a[:, 0] != 0) * 1 + (a[:, 1] != 0) * 2 + (a[:, 2] != 0) * 4)
    return np.ascontiguousarray(a, dtype=np.uint8)


class OracleEnv:
    """Host twin of VecDroneEnv driven by the C restatement."""

    def __init__(self, num_envs: int, *, precision: str = "f64", config: EnvConfig | None = None,
                 env_id_base: int = 0, **switches):
        self.cfg = (config or EnvConfig()).replace(**switches)
        self._cfg = self.cfg.to_abi()
        self.n = int(num_envs)
        self.precision = precision
        dt = np.float64 if precision == "f64" else np.float32
        self.dtype = dt
        for f in FLOAT_FIELDS:
            setattr(self, f, np.zeros(self.n, dtype=dt))
        self.status = np.zeros(self.n, dtype=np.uint8)
        self.steps = np.zeros(self.n, dtype=np.int32)
        self.episode = np.zeros(self.n, dtype=np.int32)
        self.env_id_base = env_id_base
        c = self.cfg
        self.x[:] = c.drone_start_x
        self.y[:] = c.drone_start_y
        self.fuel[:] = c.max_fuel
        self.px[:] = c.platform_start_x
        self.py[:] = c.platform_start_y

    def _state(self):
        return abi.DDState(*[_p(getattr(self, f)) for f in FLOAT_FIELDS], _p(self.status), _p(self.steps),
                           _p(self.episode), self.env_id_base, 0 if self.precision == "f32" else 1, 0)

    def step(self, actions):
        a = bitmask(actions)
        assert a.shape == (self.n,)
        reward = np.zeros(self.n, dtype=self.dtype)
        done = np.zeros(self.n, dtype=np.uint8)
        obs = np.zeros((self.n, 15), dtype=np.float32)
        obs64 = np.zeros((self.n, 15), dtype=np.float64)
        st = self._state()
        lib().ora_step(ctypes.byref(self._cfg), ctypes.byref(st), _p(a), _p(reward), _p(done), _p(obs),
                       _p(obs64), self.n)
        return obs, reward, done.astype(bool), obs64

    def step_shaped(self, actions, hist, max_steps=0, mode="notebook"):
        """step() plus the notebooks' reward: PPO's (``mode="notebook"``;
        `hist` is a [2, n] float64 array updated in place) or REINFORCE's
        (``mode="reinforce"``; `hist` is not read).  Returns obs, reward, done,
        obs64, shaped, shaped_done."""
        a = bitmask(actions)
        if mode == "notebook" or hist is not None:
            assert hist.shape == (2, self.n) and hist.dtype == np.float64 and hist.flags.c_contiguous
        reward = np.zeros(self.n, dtype=self.dtype)
        shaped = np.zeros(self.n, dtype=self.dtype)
        done = np.zeros(self.n, dtype=np.uint8)
        sdone = np.zeros(self.n, dtype=np.uint8)
        obs = np.zeros((self.n, 15), dtype=np.float32)
        obs64 = np.zeros((self.n, 15), dtype=np.float64)
        st = self._state()
        lib().ora_step_shaped(ctypes.byref(self._cfg), ctypes.byref(st), _p(a), _p(reward), _p(done), _p(obs),
                              _p(obs64), _p(hist) if hist is not None else None, _p(shaped), _p(sdone),
                              int(max_steps), 1 if mode == "reinforce" else 0, self.n)
        return obs, reward, done.astype(bool), obs64, shaped, sdone.astype(bool)

    def reset(self, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        obs = np.zeros((self.n, 15), dtype=np.float32)
        obs64 = np.zeros((self.n, 15), dtype=np.float64)
        st = self._state()
        lib().ora_reset(ctypes.byref(self._cfg), ctypes.byref(st), _p(m), _p(obs), _p(obs64), self.n)
        return obs, obs64

    def get_state(self):
        obs = np.zeros((self.n, 15), dtype=np.float32)
        obs64 = np.zeros((self.n, 15), dtype=np.float64)
        st = self._state()
        lib().ora_write_obs(ctypes.byref(self._cfg), ctypes.byref(st), _p(obs), _p(obs64), self.n)
        return obs, obs64

    def probe(self, actions):
        """Post-update (x, y, speed, angle, bottom x, bottom y, vx, vy) of every
        lane stepped with `actions`, as [n, 8] float64; the state is unchanged."""
        a = bitmask(actions)
        q = np.zeros((self.n, 8), dtype=np.float64)
        lib().ora_probe(ctypes.byref(self._cfg), ctypes.byref(self._state()), _p(a), _p(q), self.n)
        return q

    def get_info(self):
        d = np.zeros(self.n)
        s = np.zeros(self.n)
        st = self._state()
        lib().ora_get_info(ctypes.byref(self._cfg), ctypes.byref(st), _p(d), _p(s), self.n)
        return d, s

    def state_dict(self):
        d = {f: getattr(self, f).copy() for f in FLOAT_FIELDS}
        d.update(status=self.status.copy(), steps=self.steps.copy(), episode=self.episode.copy())
        return d

    def load_state_dict(self, d):
        for k, v in d.items():
            getattr(self, k)[:] = v


def gae(rewards, values, dones, gamma=0.99, lam=0.95):
    """compute_gae per column of [T, n] float32 arrays (values [T+1, n])."""
    r = np.ascontiguousarray(rewards, dtype=np.float32)
    v = np.ascontiguousarray(values, dtype=np.float32)
    d = np.ascontiguousarray(dones, dtype=np.uint8)
    T, n = r.shape
    adv = np.zeros((T, n), dtype=np.float32)
    lib().ora_gae(_p(r), _p(v), _p(d), _p(adv), T, n, gamma, lam)
    return adv


def bench(config: EnvConfig, lane0: int, n: int, steps: int) -> float:
    """Run the C restatement over a config-3 style workload (CPU baseline)."""
    cfg = config.to_abi()
    return lib().ora_bench(ctypes.byref(cfg), lane0, n, steps)
