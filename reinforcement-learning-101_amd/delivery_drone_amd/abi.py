"""ctypes mirror of ``include/dronestep.h`` and the loader of ``libdronestep.so``.

The shared library is the product: HIP kernels for gfx950 behind a plain C ABI.
There is no CPU fallback anywhere in this package — if the library is missing
or cannot be loaded, :func:`lib` raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  -- must be loaded first so the library binds torch's HIP runtime

__all__ = [
    "DD_F32", "DD_F64", "DD_ACT_BITMASK", "DD_ACT_F32X3", "DD_ACT_U8X3", "DD_ACT_PHILOX",
    "DD_ST_DONE", "DD_ST_LANDED", "DD_ST_CRASHED", "DD_ST_PLAT_LEFT", "DD_OBS_DIM",
    "DD_RENDER_HUD", "DD_RENDER_GAME_OVER", "DD_MLP_F32", "DD_MLP_F16X3",
    "DD_SHAPED_PPO", "DD_SHAPED_REINFORCE", "DD_ROLLOUT_AUTO", "DD_ROLLOUT_SINGLE", "DD_ROLLOUT_SPLIT_NO_WAIT",
    "DD_ROLLOUT_FLUSHED", "DD_ROLLOUT_HELD", "DD_ROLLOUT_SPLIT", "DD_ERR_HANDOVER",
    "DDConfig", "DDState", "DDStepIO", "DDRolloutIO", "DDMlpParams", "DDMlpIO", "DDPolicyRolloutIO", "lib", "load", "library_path", "check",
    "NativeLibraryError",
]

DD_ABI_VERSION = 12
DD_F32, DD_F64 = 0, 1
DD_ACT_BITMASK, DD_ACT_F32X3, DD_ACT_U8X3, DD_ACT_PHILOX = 0, 1, 2, 3
DD_ST_DONE, DD_ST_LANDED, DD_ST_CRASHED, DD_ST_PLAT_LEFT = 1, 2, 4, 8
DD_OBS_DIM = 15
DD_RENDER_HUD, DD_RENDER_GAME_OVER = 1, 2
DD_MLP_F32, DD_MLP_F16X3 = 0, 1
DD_SHAPED_PPO, DD_SHAPED_REINFORCE = 0, 1
DD_ROLLOUT_AUTO, DD_ROLLOUT_SINGLE, DD_ROLLOUT_SPLIT_NO_WAIT = 0, 1, 2
DD_ROLLOUT_FLUSHED, DD_ROLLOUT_HELD, DD_ROLLOUT_SPLIT = 16, 17, 18
DD_ERR_HANDOVER = 1
DD_MEM_DEFAULT, DD_MEM_CONTIGUOUS = 0, 1

_D = ctypes.c_double
_I = ctypes.c_int32


class DDConfig(ctypes.Structure):
    """``DDConfig`` (include/dronestep.h); field order is the ABI."""

    _fields_ = [
        ("gravity", _D), ("drag", _D), ("angular_drag", _D),
        ("main_thrust_power", _D), ("side_thrust_power", _D),
        ("fuel_main", _D), ("fuel_side", _D), ("max_fuel", _D),
        ("drone_half_height", _D), ("dt", _D),
        ("platform_half_width", _D), ("platform_half_height", _D),
        ("platform_speed", _D), ("platform_min_x", _D), ("platform_max_x", _D),
        ("max_landing_velocity", _D), ("max_landing_angle", _D),
        ("world_width", _D), ("world_height", _D), ("oob_margin", _D), ("ground_level", _D),
        ("wind_x", _D), ("wind_y", _D),
        ("reward_step", _D), ("reward_landing", _D), ("reward_crash", _D),
        ("reward_out_of_fuel", _D), ("reward_out_of_bounds", _D),
        ("shaping_offset", _D), ("shaping_scale", _D),
        ("vel_scale", _D), ("angle_scale", _D),
        ("drone_start_x", _I), ("drone_start_y", _I),
        ("drone_x_min", _I), ("drone_x_max", _I),
        ("drone_y_min", _I), ("drone_y_max", _I),
        ("platform_start_x", _I), ("platform_start_y", _I),
        ("platform_x_lo", _I), ("platform_x_hi", _I),
        ("platform_y_lo", _I), ("platform_y_hi", _I),
        ("wind_enabled", _I), ("platform_moving", _I),
        ("randomize_drone", _I), ("randomize_platform", _I),
        ("auto_reset", _I), ("_pad", _I),
        ("seed", ctypes.c_uint64),
    ]


class DDState(ctypes.Structure):
    _fields_ = [
        ("x", ctypes.c_void_p), ("y", ctypes.c_void_p), ("vx", ctypes.c_void_p),
        ("vy", ctypes.c_void_p), ("angle", ctypes.c_void_p), ("omega", ctypes.c_void_p),
        ("fuel", ctypes.c_void_p), ("px", ctypes.c_void_p), ("py", ctypes.c_void_p),
        ("total_reward", ctypes.c_void_p),
        ("status", ctypes.c_void_p), ("steps", ctypes.c_void_p), ("episode", ctypes.c_void_p),
        ("env_id_base", ctypes.c_int64), ("precision", _I), ("_pad", _I),
    ]


class DDStepIO(ctypes.Structure):
    _fields_ = [
        ("actions", ctypes.c_void_p), ("action_format", _I), ("_pad", _I),
        ("reward", ctypes.c_void_p), ("done", ctypes.c_void_p), ("obs", ctypes.c_void_p),
        ("done_idx", ctypes.c_void_p), ("done_count", ctypes.c_void_p),
        ("shaped_hist", ctypes.c_void_p), ("shaped_reward", ctypes.c_void_p), ("shaped_done", ctypes.c_void_p),
        ("max_steps", _I), ("shaped_mode", _I), ("state_out", ctypes.c_void_p),
    ]


class DDRolloutIO(ctypes.Structure):
    _fields_ = [
        ("actions", ctypes.c_void_p), ("action_format", _I), ("frames", _I),
        ("reward", ctypes.c_void_p), ("done", ctypes.c_void_p), ("obs", ctypes.c_void_p),
        ("action_seed", ctypes.c_uint64), ("action_step", ctypes.c_int64),
        ("shaped_hist", ctypes.c_void_p), ("engine_reward", ctypes.c_void_p), ("engine_done", ctypes.c_void_p),
        ("max_steps", _I), ("shaped_mode", _I), ("kernel", _I), ("_pad", _I),
    ]


class DDMlpParams(ctypes.Structure):
    _fields_ = [(name, ctypes.c_void_p) for name in (
        "w0", "b0", "ln1_w", "ln1_b", "w3", "b3", "ln4_w", "ln4_b",
        "w6", "b6", "ln7_w", "ln7_b", "w9", "b9")] + [("out_dim", _I), ("ln_eps", ctypes.c_float)]


class DDMlpIO(ctypes.Structure):
    _fields_ = [
        ("obs", ctypes.c_void_p), ("out", ctypes.c_void_p), ("actions", ctypes.c_void_p),
        ("log_prob", ctypes.c_void_p), ("seed", ctypes.c_uint64), ("step", ctypes.c_int64),
        ("env_id_base", ctypes.c_int64),
    ]


class DDPolicyRolloutIO(ctypes.Structure):
    _fields_ = [
        ("obs0", ctypes.c_void_p), ("obs_final", ctypes.c_void_p), ("obs", ctypes.c_void_p),
        ("actions", ctypes.c_void_p), ("log_prob", ctypes.c_void_p),
        ("reward", ctypes.c_void_p), ("done", ctypes.c_void_p),
        ("seed", ctypes.c_uint64), ("step", ctypes.c_int64), ("frames", _I), ("max_steps", _I),
        ("shaped_hist", ctypes.c_void_p), ("engine_reward", ctypes.c_void_p), ("engine_done", ctypes.c_void_p),
        ("shaped_mode", _I), ("_pad", _I),
    ]


#: every symbol include/dronestep.h declares, with its ctypes signature
EXPORTS = {
    "dd_config_default": (None, [ctypes.POINTER(DDConfig)]),
    "dd_step": (ctypes.c_int, [ctypes.POINTER(DDConfig), ctypes.POINTER(DDState),
                               ctypes.POINTER(DDStepIO), ctypes.c_int64, ctypes.c_void_p]),
    "dd_rollout": (ctypes.c_int, [ctypes.POINTER(DDConfig), ctypes.POINTER(DDState),
                                  ctypes.POINTER(DDRolloutIO), ctypes.c_int64, ctypes.c_void_p]),
    "dd_rollout_kernel": (ctypes.c_int, [ctypes.POINTER(DDConfig), ctypes.POINTER(DDState),
                                         ctypes.POINTER(DDRolloutIO), ctypes.c_int64]),
    "dd_device_errors": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint32), _I]),
    "dd_reset": (ctypes.c_int, [ctypes.POINTER(DDConfig), ctypes.POINTER(DDState), ctypes.c_void_p,
                                ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    "dd_shaped_reset": (ctypes.c_int, [ctypes.POINTER(DDConfig), ctypes.POINTER(DDState), ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    "dd_write_obs": (ctypes.c_int, [ctypes.POINTER(DDConfig), ctypes.POINTER(DDState), ctypes.c_void_p,
                                    ctypes.c_int64, ctypes.c_void_p]),
    "dd_get_info": (ctypes.c_int, [ctypes.POINTER(DDConfig), ctypes.POINTER(DDState), ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    "dd_gae": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.c_int64, ctypes.c_int64, ctypes.c_double, ctypes.c_double, ctypes.c_void_p]),
    "dd_compact_workspace": (ctypes.c_int64, [ctypes.c_int64]),
    "dd_compact": (ctypes.c_int, [ctypes.c_void_p, _I, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    "dd_mlp_packed_floats": (ctypes.c_int64, []),
    "dd_mlp_pack": (ctypes.c_int, [ctypes.POINTER(DDMlpParams), _I, ctypes.c_void_p, ctypes.c_void_p]),
    "dd_mlp_forward": (ctypes.c_int, [ctypes.c_void_p, _I, _I, ctypes.POINTER(DDMlpIO), ctypes.c_int64,
                                      ctypes.c_void_p]),
    "dd_policy_rollout": (ctypes.c_int, [ctypes.POINTER(DDConfig), ctypes.POINTER(DDState), ctypes.c_void_p, _I,
                                         ctypes.POINTER(DDPolicyRolloutIO), ctypes.c_int64, ctypes.c_void_p]),
    "dd_render": (ctypes.c_int, [ctypes.POINTER(DDConfig), ctypes.POINTER(DDState), ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, _I,
                                 ctypes.c_void_p]),
    "dd_step_bytes_per_env": (ctypes.c_int64, [_I, _I, _I]),
    "dd_error_string": (ctypes.c_char_p, [ctypes.c_int]),
    "dd_abi_version": (ctypes.c_int, []),
    "dd_build_info": (ctypes.c_char_p, []),
    "dd_selftest_sqrt": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "dd_stamp": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "dd_wall_clock_khz": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "dd_device_alloc": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint64, _I]),
    "dd_device_free": (ctypes.c_int, [ctypes.c_void_p]),
}

#: symbols a timing-only lab build (tools/build_variants.sh) or an older
#: committed source built for an A/B run may lack
_LAB_OPTIONAL = ("dd_build_info", "dd_selftest_sqrt", "dd_rollout_kernel", "dd_device_errors", "dd_stamp",
                 "dd_wall_clock_khz", "dd_device_alloc", "dd_device_free")


class NativeLibraryError(RuntimeError):
    """The HIP extension is missing, stale or failed a call."""


_LIB = None
_LOCK = threading.Lock()


def library_path() -> str:
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "_native", "libdronestep.so")


def load(path: str, *, abi_versions=None) -> ctypes.CDLL:
    """Load a build of the library at ``path`` and bind the header's signatures.
    ``abi_versions``: the versions accepted (default: this header's only); A/B
    labs pass the two sides of a version bump whose signatures are unchanged."""
    if not os.path.exists(path):
        raise NativeLibraryError(
            f"HIP extension not built: {path} is missing. "
            "Run `python -c 'import __graft_entry__ as g; g.build()'` from the repo root.")
    try:
        handle = ctypes.CDLL(path)
    except OSError as exc:  # pragma: no cover - depends on the box
        raise NativeLibraryError(f"cannot load {path}: {exc}") from exc
    for name, (restype, argtypes) in EXPORTS.items():
        if name in _LAB_OPTIONAL and not hasattr(handle, name):
            continue
        fn = getattr(handle, name)
        fn.restype = restype
        fn.argtypes = argtypes
    if handle.dd_abi_version() not in (abi_versions or (DD_ABI_VERSION,)):
        raise NativeLibraryError(f"{path}: ABI version mismatch; rebuild it")
    return handle


def lib() -> ctypes.CDLL:
    """The product library ``_native/libdronestep.so`` (built by
    ``__graft_entry__.build()``); raises if it is absent."""
    global _LIB
    if _LIB is None:
        with _LOCK:
            if _LIB is None:
                _LIB = load(library_path())
    return _LIB


def check(code: int, what: str) -> None:
    """Raise :class:`NativeLibraryError` for a nonzero HIP status."""
    if code != 0:
        msg = lib().dd_error_string(code)
        raise NativeLibraryError(f"{what} failed: HIP error {code} ({msg.decode() if msg else '?'})")
