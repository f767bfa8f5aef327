"""Generalised advantage estimation over rollout buffers (``dd_gae``).

The batched form of the notebooks' ``compute_gae`` (Actor_Critic_PPO.ipynb:
733-787): the reference runs it once per episode on a 1-D tensor; here every
lane of a ``[T, N]`` rollout is one column, scanned backwards by one GPU lane,
with ``done[t]`` cutting the recursion exactly as the notebook's mask does.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import torch

from . import abi

__all__ = ["gae"]


def gae(rewards: torch.Tensor, values: torch.Tensor, dones: torch.Tensor, gamma: float = 0.99,
        lambda_: float = 0.95, *, returns: bool = True,
        out: Optional[Tuple[torch.Tensor, Optional[torch.Tensor]]] = None):
    """Advantages (and returns = advantages + values[:T]) of a ``[T, N]`` rollout.

    ``values`` is ``[T + 1, N]`` (row T = bootstrap) or ``[T, N]`` (bootstrap
    0, as compute_gae appends).  All tensors live on one GPU; rewards/values
    are float32, dones bool/uint8 (nonzero = done).
    """
    if rewards.dim() != 2:
        raise ValueError("rewards must be [T, N]")
    T, n = rewards.shape
    dev = rewards.device
    if dev.type != "cuda":
        raise ValueError("gae runs on the GPU; move the rollout to a CUDA/HIP device")
    r = rewards.to(torch.float32).contiguous()
    v = values.to(device=dev, dtype=torch.float32)
    if v.dim() == 1 and n == 1:
        v = v[:, None]
    if v.shape == (T, n):
        v = torch.cat([v, v.new_zeros(1, n)], dim=0)
    if v.shape != (T + 1, n):
        raise ValueError(f"values must be [T+1, N] or [T, N], got {tuple(values.shape)} for T={T}, N={n}")
    v = v.contiguous()
    d = dones.to(device=dev)
    d = (d.view(torch.uint8) if d.dtype == torch.bool else (d != 0).to(torch.uint8)).contiguous()
    if d.shape != (T, n):
        raise ValueError(f"dones must be [T, N], got {tuple(dones.shape)}")
    if out is not None:
        adv, ret = out

        def _check(t, what):
            if (not isinstance(t, torch.Tensor) or t.dtype != torch.float32 or tuple(t.shape) != (T, n)
                    or not t.is_contiguous() or t.device != dev):
                raise ValueError(f"out {what} must be a contiguous float32 tensor of shape {(T, n)} on {dev}")

        _check(adv, "advantages")
        if returns:
            if ret is None:
                raise ValueError("out=(adv, None) with returns=True: pass a returns buffer")
            _check(ret, "returns")
        else:
            ret = None
    else:
        adv = torch.empty(T, n, dtype=torch.float32, device=dev)
        ret = torch.empty_like(adv) if returns else None
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    abi.check(abi.lib().dd_gae(r.data_ptr(), v.data_ptr(), d.data_ptr(), adv.data_ptr(),
                               ret.data_ptr() if ret is not None else None, T, n, float(gamma), float(lambda_),
                               stream), "dd_gae")
    return (adv, ret) if returns else adv
