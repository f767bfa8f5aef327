"""MI355X-native vectorised delivery-drone environment.

The per-frame step of vedant-jumle/reinforcement-learning-101's
``delivery_drone/game`` (physics, reward, termination) as HIP kernels for
gfx950 behind a C ABI (``include/dronestep.h``), with a gym-style batched
surface (:class:`VecDroneEnv`) and the reference's per-game APIs
(:class:`DroneGameClient`, :class:`DroneGame`) on top; the notebooks'
policy / value networks (:class:`MlpNet`, f32 MFMA) and GAE (:func:`gae`)
for on-device collection.
"""
from .config import EnvConfig
from .vec_env import OBS_KEYS, StepInfo, VecDroneEnv
from .compat import DroneGame, DroneGameClient, DroneState, action_bits
from .sharding import dist_env, gather_obs, shard_bounds
from .gae import gae
from .policy import MlpNet

__all__ = [
    "EnvConfig", "VecDroneEnv", "StepInfo", "OBS_KEYS",
    "DroneGame", "DroneGameClient", "DroneState", "action_bits",
    "shard_bounds", "dist_env", "gather_obs", "gae", "MlpNet",
]
__version__ = "0.1.0"
