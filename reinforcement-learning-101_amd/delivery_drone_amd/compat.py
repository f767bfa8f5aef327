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

from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import torch

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
    """Host-side readback of single lanes of a VecDroneEnv."""

    def __init__(self, env: VecDroneEnv):
        self.env = env

    def obs_dict(self, g: int) -> dict:
        e = self.env
        row = e.obs[g].tolist()
        return _state_dict(row, int(e.steps[g].item()))

    def info(self, g: int) -> dict:
        e = self.env
        info = e.get_info()
        return {
            "steps": int(e.steps[g].item()),
            "total_reward": float(e.total_reward[g].item()),
            "episode": int(e.episode[g].item()),
            "fuel_remaining": float(e.fuel[g].item()),
            "distance_to_platform": float(info["distance_to_platform"][g].item()),
            "speed": float(info["speed"][g].item()),
            "angle": float(e.angle[g].item()),
        }

    def step(self, g: int, action: Dict) -> Tuple[dict, float, bool, dict]:
        e = self.env
        was_done = bool(e.status[g].item() & 1)
        a = torch.tensor([action_bits(action)], dtype=torch.uint8, device=e.device)
        e.step(a, lanes=slice(g, g + 1))
        info = self.info(g)
        if was_done and not e.config.auto_reset:
            info["needs_reset"] = True  # game_engine.py:107-111
        return self.obs_dict(g), float(e.reward[g].item()), bool(e.done[g].item()), info

    def reset(self, g: int) -> dict:
        self.env.reset(lanes=slice(g, g + 1))
        return self.obs_dict(g)

    def get_state(self, g: int) -> dict:
        self.env.get_state()
        return self.obs_dict(g)


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

    ``render_mode`` must be None: rendering is out of scope for this path.
    Defaults to ``precision="f64"`` so a single game tracks the reference's
    double-precision trajectory.
    """

    def __init__(self, render_mode=None, randomize_drone: bool = False, randomize_platform: bool = True, *,
                 seed: int = 0, device=None, precision: str = "f64", config=None, env_id: int = 0):
        if render_mode is not None:
            raise NotImplementedError("rendering is out of scope; use render_mode=None")
        self.render_mode = None
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
        return None

    def close(self):
        pass
