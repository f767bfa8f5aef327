"""World constants of the delivery-drone game as one frozen dataclass.

Defaults are the values of the reference's module constants
(``delivery_drone/game/config.py:17-68``); the reference changes behaviour by
editing that module (wind, moving platform, spawn ranges), here by building an
:class:`EnvConfig` with other values.  :meth:`EnvConfig.to_abi` produces the
``DDConfig`` struct the kernels read from their kernarg segment.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass

from . import abi

# config.py:3-4, 32-34 — window and platform geometry the derived values use
WINDOW_WIDTH = 800
WINDOW_HEIGHT = 600
DRONE_WIDTH, DRONE_HEIGHT = 40, 20
PLATFORM_WIDTH, PLATFORM_HEIGHT = 100, 20


@dataclass(frozen=True)
class EnvConfig:
    # physics (config.py:18-29)
    gravity: float = 0.3
    drag: float = 0.99
    angular_drag: float = 0.95
    main_thrust_power: float = 0.6
    side_thrust_power: float = 0.3
    fuel_main: float = 2.0
    fuel_side: float = 1.0
    max_fuel: float = 1000.0
    drone_half_height: float = DRONE_HEIGHT / 2  # Drone.get_bottom_center (drone.py:136)
    dt: float = 1.0
    # platform (config.py:32-36, platform.py:20-29)
    platform_half_width: float = PLATFORM_WIDTH / 2
    platform_half_height: float = PLATFORM_HEIGHT / 2
    platform_speed: float = 1.0
    platform_min_x: float = PLATFORM_WIDTH // 2
    platform_max_x: float = WINDOW_WIDTH - PLATFORM_WIDTH // 2
    # landing (config.py:39-40)
    max_landing_velocity: float = 3.0
    max_landing_angle: float = 20.0
    # bounds (config.py:45, game_engine.py:254)
    world_width: float = WINDOW_WIDTH
    world_height: float = WINDOW_HEIGHT
    oob_margin: float = 50
    ground_level: float = WINDOW_HEIGHT - 50
    # wind (config.py:48-49, game_engine.py:56-57, 121-123)
    wind_enabled: bool = False
    wind_x: float = 0.0
    wind_y: float = 0.0
    platform_moving: bool = False  # config.py:50
    # rewards (config.py:54-58, game_engine.py:214)
    reward_step: float = -0.1
    reward_landing: float = 100.0
    reward_crash: float = -100.0
    reward_out_of_fuel: float = -50.0
    reward_out_of_bounds: float = -50.0
    shaping_offset: float = 500
    shaping_scale: float = 5000
    # observation scales (game_engine.py:155-171)
    vel_scale: float = 10.0
    angle_scale: float = 180.0
    # spawn (config.py:61-68, game_engine.py:66-85)
    drone_start_x: int = WINDOW_WIDTH // 2
    drone_start_y: int = 100
    drone_x_min: int = 100
    drone_x_max: int = 700
    drone_y_min: int = 50
    drone_y_max: int = 250
    platform_start_x: int = WINDOW_WIDTH // 2
    platform_start_y: int = WINDOW_HEIGHT - 100
    platform_x_lo: int = PLATFORM_WIDTH // 2 + 50
    platform_x_hi: int = WINDOW_WIDTH - PLATFORM_WIDTH // 2 - 50
    platform_y_lo: int = 100
    platform_y_hi: int = 550
    # switches (DroneGame(randomize_drone=False, randomize_platform=True), game_engine.py:14)
    randomize_drone: bool = False
    randomize_platform: bool = True
    auto_reset: bool = False
    seed: int = 0

    def replace(self, **kw) -> "EnvConfig":
        return dataclasses.replace(self, **kw)

    def to_abi(self) -> abi.DDConfig:
        c = abi.DDConfig()
        for f in dataclasses.fields(self):
            v = getattr(self, f.name)
            if f.name == "seed":
                v = int(v) & 0xFFFFFFFFFFFFFFFF
            elif isinstance(v, bool):
                v = int(v)
            setattr(c, f.name, v)
        return c

    def validate(self) -> None:
        if self.drone_x_max < self.drone_x_min or self.drone_y_max < self.drone_y_min:
            raise ValueError("drone spawn range is empty")
        if self.platform_x_hi <= self.platform_x_lo or self.platform_y_hi <= self.platform_y_lo:
            raise ValueError("platform spawn range is empty (the upper bound is exclusive)")
        for name in ("world_width", "world_height", "vel_scale", "angle_scale", "max_fuel", "shaping_scale"):
            if getattr(self, name) == 0:
                raise ValueError(f"{name} must be nonzero (it is a divisor)")
