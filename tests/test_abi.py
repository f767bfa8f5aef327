"""CPU: the product library loads, exports the header's ABI, and validates
arguments — without touching a GPU (no compute calls here)."""
import ctypes
import dataclasses
import os
import re
import subprocess

import pytest

from delivery_drone_amd import abi
from delivery_drone_amd.config import EnvConfig

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "dronestep.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dd_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_what_abi_binds():
    assert header_functions() == sorted(abi.EXPORTS)


def test_library_exports_every_header_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", abi.library_path()], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (dd_[a-z0-9_]+)$", out, flags=re.M))
    missing = set(header_functions()) - exported
    assert not missing, missing


def test_library_is_gfx950_code():
    blob = open(abi.library_path(), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # the offload bundle's target id


def test_library_loads_and_reports_abi():
    lib = abi.lib()
    assert lib.dd_abi_version() == abi.DD_ABI_VERSION


def test_c_defaults_equal_envconfig_defaults():
    """dd_config_default (C) vs EnvConfig (Python): also checks the ctypes
    struct layout against the C one field by field."""
    c = abi.DDConfig()
    abi.lib().dd_config_default(ctypes.byref(c))
    py = EnvConfig().to_abi()
    for name, _ in abi.DDConfig._fields_:
        assert getattr(c, name) == getattr(py, name), name
    assert ctypes.sizeof(abi.DDConfig) == 32 * 8 + 18 * 4 + 8


def test_envconfig_matches_reference_constants():
    c = EnvConfig()
    assert (c.gravity, c.drag, c.angular_drag) == (0.3, 0.99, 0.95)
    assert (c.main_thrust_power, c.side_thrust_power, c.max_fuel) == (0.6, 0.3, 1000.0)
    assert (c.platform_x_lo, c.platform_x_hi, c.platform_y_lo, c.platform_y_hi) == (100, 700, 100, 550)
    assert (c.drone_x_min, c.drone_x_max, c.drone_y_min, c.drone_y_max) == (100, 700, 50, 250)
    assert (c.ground_level, c.oob_margin, c.max_landing_velocity, c.max_landing_angle) == (550, 50, 3.0, 20.0)
    assert c.randomize_platform and not c.randomize_drone and not c.auto_reset


def test_envconfig_validation():
    with pytest.raises(ValueError):
        EnvConfig(platform_x_hi=100).validate()
    with pytest.raises(ValueError):
        EnvConfig(world_width=0).validate()
    cfg = EnvConfig(seed=2**64 + 5).to_abi()
    assert cfg.seed == 5
    assert dataclasses.replace(EnvConfig(), auto_reset=True).to_abi().auto_reset == 1


def _state(n_ptr=1, precision=abi.DD_F32):
    p = ctypes.c_void_p(n_ptr)
    return abi.DDState(p, p, p, p, p, p, p, p, p, p, p, p, p, 0, precision, 0)


def test_argument_errors_return_invalid_value_without_gpu():
    lib = abi.lib()
    cfg = EnvConfig().to_abi()
    io = abi.DDStepIO()
    io.actions = io.reward = io.done = 1
    EINVAL = 1  # hipErrorInvalidValue
    assert lib.dd_step(None, ctypes.byref(_state()), ctypes.byref(io), 4, None) == EINVAL
    assert lib.dd_step(ctypes.byref(cfg), ctypes.byref(_state(precision=7)), ctypes.byref(io), 4, None) == EINVAL
    assert lib.dd_step(ctypes.byref(cfg), ctypes.byref(_state()), ctypes.byref(io), -1, None) == EINVAL
    assert lib.dd_step(ctypes.byref(cfg), ctypes.byref(_state()), ctypes.byref(io), 2**31, None) == EINVAL
    bad = abi.DDState()  # null pointers
    assert lib.dd_step(ctypes.byref(cfg), ctypes.byref(bad), ctypes.byref(io), 4, None) == EINVAL
    io.action_format = 9
    assert lib.dd_step(ctypes.byref(cfg), ctypes.byref(_state()), ctypes.byref(io), 4, None) == EINVAL
    io.action_format = 0
    io.done_idx = 8  # done_idx without done_count
    assert lib.dd_step(ctypes.byref(cfg), ctypes.byref(_state()), ctypes.byref(io), 4, None) == EINVAL
    assert lib.dd_reset(ctypes.byref(cfg), ctypes.byref(bad), None, None, 4, None) == EINVAL
    assert lib.dd_write_obs(ctypes.byref(cfg), ctypes.byref(_state()), None, 4, None) == EINVAL
    assert lib.dd_reset(ctypes.byref(cfg), ctypes.byref(bad), None, None, 0, None) == 0  # empty batch
    assert lib.dd_compact(None, 0, None, None, None, 4, None) == EINVAL
    rio = abi.DDRolloutIO()
    rio.frames = 4
    rio.action_format = 0  # bitmask needs an action buffer
    rio.reward = rio.done = 8
    assert lib.dd_rollout(ctypes.byref(cfg), ctypes.byref(_state()), ctypes.byref(rio), 4, None) == EINVAL
    rio.action_format = 4
    assert lib.dd_rollout(ctypes.byref(cfg), ctypes.byref(_state()), ctypes.byref(rio), 4, None) == EINVAL
    rio.action_format, rio.frames = 3, -1
    assert lib.dd_rollout(ctypes.byref(cfg), ctypes.byref(_state()), ctypes.byref(rio), 4, None) == EINVAL
    rio.frames = 4
    rio.engine_reward = 8  # engine outputs: both or neither, and only in notebook (shaped) mode
    assert lib.dd_rollout(ctypes.byref(cfg), ctypes.byref(_state()), ctypes.byref(rio), 4, None) == EINVAL
    rio.engine_done = 8
    assert lib.dd_rollout(ctypes.byref(cfg), ctypes.byref(_state()), ctypes.byref(rio), 4, None) == EINVAL
    rio.engine_reward = rio.engine_done = None
    rio.shaped_mode = 2  # DD_SHAPED_PPO or DD_SHAPED_REINFORCE
    assert lib.dd_rollout(ctypes.byref(cfg), ctypes.byref(_state()), ctypes.byref(rio), 4, None) == EINVAL
    rio.shaped_mode = abi.DD_SHAPED_REINFORCE  # engine outputs next to the REINFORCE reward: fine
    rio.kernel = 3  # DD_ROLLOUT_AUTO / _SINGLE / _SPLIT_NO_WAIT
    assert lib.dd_rollout(ctypes.byref(cfg), ctypes.byref(_state()), ctypes.byref(rio), 4, None) == EINVAL
    rio.kernel = abi.DD_ROLLOUT_AUTO
    rio.shaped_mode = abi.DD_SHAPED_PPO
    rio.frames = 0  # nothing to do
    assert lib.dd_rollout(ctypes.byref(cfg), ctypes.byref(_state()), ctypes.byref(rio), 4, None) == 0
    io.done_idx = None
    io.action_format = 3  # Philox actions are rollout-only
    assert lib.dd_step(ctypes.byref(cfg), ctypes.byref(_state()), ctypes.byref(io), 4, None) == EINVAL
    io.action_format = 0
    io.shaped_reward = 8  # PPO mode: the three shaped pointers together or none
    assert lib.dd_step(ctypes.byref(cfg), ctypes.byref(_state()), ctypes.byref(io), 4, None) == EINVAL
    io.shaped_mode = abi.DD_SHAPED_REINFORCE  # REINFORCE: reward and done, no history
    assert lib.dd_step(ctypes.byref(cfg), ctypes.byref(_state()), ctypes.byref(io), 4, None) == EINVAL
    io.shaped_mode = 5
    io.shaped_done = 8
    assert lib.dd_step(ctypes.byref(cfg), ctypes.byref(_state()), ctypes.byref(io), 4, None) == EINVAL
    assert lib.dd_error_string(EINVAL)


def test_rollout_kernel_choice_without_gpu():
    """dd_rollout_kernel names the kernel dd_rollout would launch (host logic
    only; the split kernel needs the device's CU count, so it is not chosen
    here)."""
    lib = abi.lib()
    cfg = EnvConfig().to_abi()
    rio = abi.DDRolloutIO()
    rio.frames, rio.reward, rio.done = 4, 8, 8
    rio.action_format = abi.DD_ACT_PHILOX
    st = _state()
    assert lib.dd_rollout_kernel(ctypes.byref(cfg), ctypes.byref(st), ctypes.byref(rio), 8) == abi.DD_ROLLOUT_HELD
    rio.obs = 16 + 4  # rows not 16-byte aligned: the flushed path
    assert lib.dd_rollout_kernel(ctypes.byref(cfg), ctypes.byref(st), ctypes.byref(rio), 8) == abi.DD_ROLLOUT_FLUSHED
    assert lib.dd_rollout_kernel(ctypes.byref(cfg), ctypes.byref(st), ctypes.byref(rio), 6) == abi.DD_ROLLOUT_FLUSHED
    assert lib.dd_rollout_kernel(None, ctypes.byref(st), ctypes.byref(rio), 8) == -1
    assert lib.dd_rollout_kernel(ctypes.byref(cfg), ctypes.byref(st), ctypes.byref(rio), 0) == -1
    assert lib.dd_device_errors(None, 0) == 1  # EINVAL: no output


def test_policy_rollout_argument_errors_without_gpu():
    lib = abi.lib()
    cfg = EnvConfig().to_abi()
    EINVAL = 1
    assert ctypes.sizeof(abi.DDPolicyRolloutIO) == 7 * 8 + 8 + 8 + 4 + 4 + 3 * 8 + 8  # the C struct's layout
    assert ctypes.sizeof(abi.DDRolloutIO) == 8 + 8 + 3 * 8 + 8 + 8 + 3 * 8 + 4 * 4
    assert ctypes.sizeof(abi.DDStepIO) == 8 + 8 + 5 * 8 + 3 * 8 + 8 + 8
    io = abi.DDPolicyRolloutIO()
    io.obs0 = io.reward = io.done = 8
    io.frames = 4

    def run(state=None, packed=16, compute=abi.DD_MLP_F16X3, n=4, c=cfg):
        st = state if state is not None else _state()
        return lib.dd_policy_rollout(ctypes.byref(c) if c is not None else None, ctypes.byref(st), packed, compute,
                                     ctypes.byref(io), n, None)

    assert run(c=None) == EINVAL
    assert run(state=abi.DDState()) == EINVAL  # null SoA pointers
    assert run(state=_state(precision=7)) == EINVAL
    assert run(n=-1) == EINVAL
    assert run(compute=5) == EINVAL
    assert run(packed=None) == EINVAL
    assert run(packed=8) == EINVAL  # packed parameters are read as 16-byte fragments
    io.obs0 = None
    assert run() == EINVAL  # frame 0's policy input is required
    io.obs0 = 8
    io.reward = None
    assert run() == EINVAL
    io.reward = 8
    io.engine_reward = 8  # engine outputs: both or neither, and only in notebook mode
    assert run() == EINVAL
    io.engine_done = 8
    assert run() == EINVAL
    io.engine_reward = io.engine_done = None
    io.frames = -1
    assert run() == EINVAL
    io.frames = 0  # nothing to do (and no final observation wanted)
    assert run() == 0
    assert run(n=0) == 0


def test_render_argument_errors_without_gpu():
    lib = abi.lib()
    cfg = EnvConfig().to_abi()
    EINVAL = 1
    st, rgb = _state(), ctypes.c_void_p(8)

    def render(c=cfg, state=st, lanes=None, count=2, n=4, out=rgb, flags=3):
        return lib.dd_render(ctypes.byref(c) if c is not None else None, ctypes.byref(state), None, lanes, count, n,
                             out, flags, None)

    assert render(c=None) == EINVAL
    assert render(count=-1) == EINVAL
    assert render(n=-1) == EINVAL
    assert render(count=5, n=4) == EINVAL  # lanes 0..4 of a 4-lane batch
    assert render(out=None) == EINVAL
    assert render(state=abi.DDState()) == EINVAL  # null SoA pointers
    assert render(state=_state(precision=7)) == EINVAL
    assert render(c=EnvConfig(world_width=802).to_abi()) == EINVAL  # rows are drawn 4 pixels at a time
    assert render(count=0) == 0  # nothing to draw


def test_byte_model():
    lib = abi.lib()
    # f32, bitmask actions, obs: reads 10*4+1+4+1, writes 9*4+4+1, obs 60
    assert lib.dd_step_bytes_per_env(abi.DD_F32, abi.DD_ACT_BITMASK, 1) == 46 + 41 + 60
    assert lib.dd_step_bytes_per_env(abi.DD_F32, abi.DD_ACT_BITMASK, 0) == 87
    assert lib.dd_step_bytes_per_env(abi.DD_F64, abi.DD_ACT_F32X3, 1) == (80 + 5 + 12) + (72 + 5) + 60
    assert lib.dd_compact_workspace(1000) == 4


def test_device_alloc_rejects_bad_arguments():
    """dd_device_alloc / dd_device_free argument checks (no HIP call reached)."""
    EINVAL = 1  # hipErrorInvalidValue
    lib = abi.lib()
    p = ctypes.c_void_p()
    assert lib.dd_device_alloc(None, 64, abi.DD_MEM_DEFAULT) == EINVAL
    assert lib.dd_device_alloc(ctypes.byref(p), 0, abi.DD_MEM_CONTIGUOUS) == EINVAL
    assert lib.dd_device_alloc(ctypes.byref(p), 64, 7) == EINVAL and p.value is None
    assert lib.dd_device_free(None) == 0


def test_memory_option_is_checked_before_the_gpu():
    from delivery_drone_amd import VecDroneEnv
    with pytest.raises(ValueError, match="memory"):
        VecDroneEnv(8, memory="pinned")


def test_no_cpu_fallback_without_gpu():
    import torch
    from delivery_drone_amd import VecDroneEnv
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        VecDroneEnv(8)


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(abi, "_LIB", None)
    monkeypatch.setattr(abi, "library_path", lambda: str(tmp_path / "nope.so"))
    with pytest.raises(abi.NativeLibraryError, match="not built"):
        abi.lib()
