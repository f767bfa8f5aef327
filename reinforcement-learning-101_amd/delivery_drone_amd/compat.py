"""Per-game facades with the reference's call signatures, backed by the GPU batch.

* :class:`DroneGameClient` — the API of ``delivery_drone/game/socket_client.py``
  (``num_games``, ``reset(game_id)``, ``step(action, game_id)``,
  ``get_state(game_id)``, ``connect/disconnect/close``, context manager, and its
  ``ValueError`` / ``RuntimeError`` behaviour), so a notebook that builds
  ``DroneGameClient()`` can switch imports.  No socket: each game is one lane of
  a :class:`VecDroneEnv`.
* :class:`DroneGame` — the in-process engine API of
  ``delivery_drone/game/game_engine.py:11-298`` (dict state, float reward,
  bool done, dict info), one lane.

Both read results back to the host on every call, like the originals; they
are for compatibility.  Throughput code calls :class:`VecDroneEnv` directly.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import torch

from . import abi
from .vec_env import OBS_KEYS, VecDroneEnv

__all__ = ["DroneState", "DroneGameClient", "DroneGame", "action_bits"]

_ACTION_KEYS = ("main_thrust", "left_thrust", "right_thrust")


@dataclass
class DroneState:
    """Same fields as ``socket_client.DroneState`` (socket_client.py:10-28)."""

    drone_x: float
    drone_y: float
    drone_vx: float
    drone_vy: float
    drone_angle: float
    drone_angular_vel: float
    drone_fuel: float
    platform_x: float
    platform_y: float
    distance_to_platform: float
    dx_to_platform: float
    dy_to_platform: float
    speed: float
    landed: bool
    crashed: bool
    steps: int


def action_bits(action: Dict) -> int:
    """``{'main_thrust', 'left_thrust', 'right_thrust'}`` -> bitmask, with the
    reference's truthiness (``bool(action.get(k, 0))``, game_engine.py:114-118)."""
    return sum(1 << k for k, name in enumerate(_ACTION_KEYS) if bool(action.get(name, 0)))


def _state_dict(obs_row, steps: int) -> dict:
    d = {k: float(v) for k, v in zip(OBS_KEYS, obs_row)}
    d["landed"] = bool(d["landed"])
    d["crashed"] = bool(d["crashed"])
    d["steps"] = int(steps)
    return d


class _Lanes:
    """Single-lane calls on a VecDroneEnv and their host readback: every
    request costs its kernel(s) plus ONE device-to-host copy of the lane's
    values (the reference returns Python objects per call)."""

    def __init__(self, env: VecDroneEnv):
        self.env = env
        self._di = torch.empty(2, dtype=env.float_dtype, device=env.device)  # distance, speed of one lane

    def _lane_kernels(self, g: int, obs: bool):
        e = self.env
        st = e._sub_state(g, 1)
        if obs:
            abi.check(e._lib.dd_write_obs(ctypes.byref(e._cfg), ctypes.byref(st), e.obs[g].data_ptr(), 1,
                                          e._stream()), "dd_write_obs")
        abi.check(e._lib.dd_get_info(ctypes.byref(e._cfg), ctypes.byref(st), self._di.data_ptr(),
                                     self._di[1:].data_ptr(), 1, e._stream()), "dd_get_info")

    def _read(self, g: int, extra: Optional[torch.Tensor] = None):
        e = self.env
        sl = slice(g, g + 1)
        f64 = torch.float64
        parts = [e.obs[g].to(f64), e.steps[sl].to(f64), e.total_reward[sl].to(f64), e.episode[sl].to(f64),
                 e.fuel[sl].to(f64), self._di.to(f64), e.angle[sl].to(f64), e.reward[sl].to(f64),
                 e.status[sl].to(f64)]
        if extra is not None:
            parts.append(extra.to(f64))
        vals = torch.cat(parts).cpu().tolist()
        self._extra = vals[24:]
        steps = int(vals[15])
        info = {"steps": steps, "total_reward": vals[16], "episode": int(vals[17]), "fuel_remaining": vals[18],
                "distance_to_platform": vals[19], "speed": vals[20], "angle": vals[21]}
        return _state_dict(vals[:15], steps), info, vals[22], int(vals[23])

    def obs_dict(self, g: int) -> dict:
        self._lane_kernels(g, obs=False)
        return self._read(g)[0]

    def info(self, g: int) -> dict:
        self._lane_kernels(g, obs=False)
        return self._read(g)[1]

    def step(self, g: int, action: Dict) -> Tuple[dict, float, bool, dict]:
        e = self.env
        a = torch.tensor([action_bits(action)], dtype=torch.uint8, device=e.device)
        was = e.status[g:g + 1].clone()  # the pre-step status, read back with the rest
        e.step(a, lanes=slice(g, g + 1))
        self._lane_kernels(g, obs=False)
        state, info, reward, status = self._read(g, was)
        if int(self._extra[0]) & 1 and not e.config.auto_reset:
            info["needs_reset"] = True  # game_engine.py:107-111
        return state, reward, bool(status & 1), info

    def reset(self, g: int) -> dict:
        self.env.reset(lanes=slice(g, g + 1))
        self._lane_kernels(g, obs=False)
        return self._read(g)[0]

    def get_state(self, g: int) -> dict:
        self._lane_kernels(g, obs=True)
        return self._read(g)[0]

    def get_state_info(self, g: int):
        """(state, done, info) of GET_STATE (socket_server.py:211-214), one readback."""
        self._lane_kernels(g, obs=True)
        state, info, _, status = self._read(g)
        return state, bool(status & 1), info


class DroneGameClient:
    """``DroneGameClient`` (socket_client.py:31-224) over a GPU batch.

    ``host``, ``port`` and ``timeout`` are accepted for signature
    compatibility and ignored.  ``num_games`` (the server's ``--num-games``)
    and the spawn switches (the server's ``--randomize-drone``,
    ``--randomize-platform``, ``--fixed-spawn``) are keyword arguments here;
    ``env`` adopts an existing :class:`VecDroneEnv`.
    """

    def __init__(self, host: str = "localhost", port: int = 5555, timeout: float = 30.0, *,
                 num_games: int = 1, env: Optional[VecDroneEnv] = None, **env_kwargs):
        self.host, self.port, self.timeout = host, port, timeout
        self._env_kwargs = env_kwargs
        self._num_games = num_games if env is None else env.num_envs
        self.env = env
        self.connected = False
        self.num_games = 1  # set by connect(), like the handshake (socket_client.py:68-70)

    def connect(self):
        if self.connected:
            return
        if self.env is None:
            self.env = VecDroneEnv(self._num_games, **self._env_kwargs)
            self.env.reset()  # the server resets every game at start (socket_server.py:147-148)
        self._lanes = _Lanes(self.env)
        self.num_games = self.env.num_envs
        self.connected = True

    def disconnect(self):
        self.connected = False

    close = disconnect

    def __enter__(self):
        self.connect()
        return self

    def __exit__(self, exc_type, exc, tb):
        self.disconnect()

    def _check_id(self, game_id: int):
        if game_id < 0 or game_id >= self.num_games:
            raise ValueError(f"Invalid game_id: {game_id}. Must be in range [0, {self.num_games})")

    def reset(self, game_id: int = 0) -> DroneState:
        if not self.connected:
            self.connect()
        self._check_id(game_id)
        return DroneState(**self._lanes.reset(game_id))

    def step(self, action: Dict[str, int], game_id: int = 0) -> Tuple[DroneState, float, bool, Dict]:
        if not self.connected:
            raise RuntimeError("Not connected to server. Call connect() or reset() first.")
        self._check_id(game_id)
        state, reward, done, info = self._lanes.step(game_id, action)
        return DroneState(**state), reward, done, info

    def get_state(self, game_id: int = 0) -> DroneState:
        if not self.connected:
            raise RuntimeError("Not connected to server")
        self._check_id(game_id)
        return DroneState(**self._lanes.get_state(game_id))


class DroneGame:
    """One game with the engine API of ``DroneGame`` (game_engine.py:11-298).

    ``render_mode`` is None (headless) or ``'rgb_array'`` (``render()``
    returns the frame as a numpy uint8 [600, 800, 3], drawn on the GPU by
    dd_render); ``'human'`` needs a pygame window and is not supported.
    Defaults to ``precision="f64"`` so a single game tracks the reference's
    double-precision trajectory.
    """

    def __init__(self, render_mode=None, randomize_drone: bool = False, randomize_platform: bool = True, *,
                 seed: int = 0, device=None, precision: str = "f64", config=None, env_id: int = 0):
        if render_mode not in (None, "rgb_array"):
            raise NotImplementedError("render_mode='human' needs a display; use None or 'rgb_array'")
        self.render_mode = render_mode
        self.env = VecDroneEnv(1, randomize_drone=randomize_drone, randomize_platform=randomize_platform,
                               auto_reset=False, seed=seed, device=device, precision=precision,
                               config=config, env_id_base=env_id)
        self._lanes = _Lanes(self.env)

    @property
    def done(self) -> bool:
        return bool(self.env.status[0].item() & 1)

    @property
    def steps(self) -> int:
        return int(self.env.steps[0].item())

    @property
    def episode(self) -> int:
        return int(self.env.episode[0].item())

    @property
    def total_reward(self) -> float:
        return float(self.env.total_reward[0].item())

    def reset(self) -> dict:
        return self._lanes.reset(0)

    def step(self, action: Dict) -> Tuple[dict, float, bool, dict]:
        return self._lanes.step(0, action)

    def get_state(self) -> dict:
        return self._lanes.get_state(0)

    def _get_info(self) -> dict:
        return self._lanes.info(0)

    def render(self):
        """game_engine.py:300-337: None headless, else the rgb_array frame."""
        if self.render_mode is None:
            return None
        return self.env.render(lanes=0)[0].cpu().numpy()

    def close(self):
        pass
