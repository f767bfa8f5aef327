"""The notebooks' policy and value networks on the GPU (``dd_mlp_forward``).

``DroneGamerBoi`` (actor) and ``DroneTeacherBoi`` (critic) of
Actor_Critic_PPO.ipynb:376-424 share one body,

    Linear(15,128) LayerNorm ReLU  Linear(128,128) LayerNorm ReLU
    Linear(128,64) LayerNorm ReLU  Linear(64,K)

with K = 3 + Sigmoid for the actor and K = 1 for the critic.  A
:class:`MlpNet` takes that state_dict (the notebooks' ``.pth`` files load with
``torch.load(path, weights_only=True)``), packs it once into the kernel's
MFMA operand order, and evaluates N observation rows per call in float32
(``compute="f32"``, the default) or with the hidden GEMMs on the f16 MFMA as
split hi/lo operand pairs (``compute="f16x3"``: about 2x faster — 65,536 rows
35.8 -> 15-18 us on MI355X — about the same end-to-end error;
include/dronestep.h ``DD_MLP_F16X3``).
The actor also does the collection loop's ``Bernoulli(probs).sample()`` and
``.log_prob(actions).sum(dim=1)`` (:857-859) in the same launch, returning the
actions as the ``dd_step`` bitmask, so a policy-driven rollout never leaves
the device.
"""
from __future__ import annotations

import ctypes
from typing import Mapping, Optional

import torch

from . import abi

__all__ = ["MlpNet", "STATE_DICT_KEYS"]

#: state_dict keys of the notebooks' nn.Sequential (``network.<i>.<param>``)
STATE_DICT_KEYS = ("0.weight", "0.bias", "1.weight", "1.bias", "3.weight", "3.bias", "4.weight", "4.bias",
                   "6.weight", "6.bias", "7.weight", "7.bias", "9.weight", "9.bias")
_SHAPES = {"0.weight": (128, 15), "0.bias": (128,), "1.weight": (128,), "1.bias": (128,),
           "3.weight": (128, 128), "3.bias": (128,), "4.weight": (128,), "4.bias": (128,),
           "6.weight": (64, 128), "6.bias": (64,), "7.weight": (64,), "7.bias": (64,)}
_COMPUTE = {"f32": abi.DD_MLP_F32, "f16x3": abi.DD_MLP_F16X3}


class MlpNet:
    """Actor (``out_dim == 3``) or critic (``out_dim == 1``) on one GPU.

    ``state_dict`` keys may carry the notebooks' ``network.`` prefix or not.
    ``ln_eps`` is nn.LayerNorm's default.  ``compute`` is ``"f32"`` or
    ``"f16x3"`` (see the module docstring).  The packed parameters stay on
    ``device``; ``library`` selects a build of libdronestep.so (tests, A/B).
    """

    def __init__(self, state_dict: Mapping[str, torch.Tensor], *, device="cuda", ln_eps: float = 1e-5,
                 compute: str = "f32", library=None):
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("MlpNet runs on the GPU (HIP); there is no CPU path")
        if self.device.index is None:  # "cuda" -> the current device, as VecDroneEnv does
            self.device = torch.device("cuda", torch.cuda.current_device())
        if compute not in _COMPUTE:
            raise ValueError(f"compute must be one of {sorted(_COMPUTE)}, got {compute!r}")
        self.compute = compute
        self._mode = _COMPUTE[compute]
        self._lib = library if library is not None else abi.lib()
        sd = {k[len("network."):] if k.startswith("network.") else k: v for k, v in state_dict.items()}
        missing = [k for k in STATE_DICT_KEYS if k not in sd]
        if missing:
            raise KeyError(f"state_dict lacks {missing}")
        for k, shape in _SHAPES.items():
            if tuple(sd[k].shape) != shape:
                raise ValueError(f"{k}: expected shape {shape}, got {tuple(sd[k].shape)}")
        k_out = sd["9.weight"].shape[0]
        if k_out not in (1, 3) or tuple(sd["9.weight"].shape) != (k_out, 64) or tuple(sd["9.bias"].shape) != (k_out,):
            raise ValueError("last layer must be Linear(64, 3) (actor) or Linear(64, 1) (critic)")
        self.out_dim = int(k_out)
        self.ln_eps = float(ln_eps)
        # keep the source tensors alive until the pack kernel has read them
        self._src = {k: torch.as_tensor(sd[k]).detach().to(device=self.device, dtype=torch.float32).contiguous()
                     for k in STATE_DICT_KEYS}
        if compute == "f16x3":
            # the hidden Linears' weights go into f16 halves x16 (kWScale) after
            # centring over their outputs (|w - mean| <= 2 max|w|): beyond the f16
            # range the hi half is inf and every probability NaN, so refuse such
            # weights here (observations must stay below 1023 as well)
            for k in ("0.weight", "3.weight", "6.weight"):
                w = self._src[k]
                if not bool(torch.isfinite(w).all()) or float(w.abs().max()) >= 65504.0 / 32:
                    raise ValueError(f"{k}: compute='f16x3' needs finite weights below 2047 in magnitude "
                                     "(the f16 range after centring and x16); use compute='f32'")
            # each LayerNorm's output x16 is split with its ReLU (mlp_core.h
            # split_pair_relu), which needs it below 2048: |gamma| sqrt(rows) +
            # |beta| bounds a LayerNorm's output
            for g, b, rows in (("1.weight", "1.bias", 128), ("4.weight", "4.bias", 128), ("7.weight", "7.bias", 64)):
                bound = float(self._src[g].abs().max()) * rows ** 0.5 * (1 + 2 ** -8) + float(self._src[b].abs().max())
                if not bound < 128.0:
                    raise ValueError(f"{g}/{b}: compute='f16x3' needs LayerNorm outputs below 128 "
                                     f"(max|weight| sqrt({rows}) + max|bias| = {bound:.4g}); use compute='f32'")
        p = abi.DDMlpParams(*[self._src[k].data_ptr() for k in STATE_DICT_KEYS], self.out_dim, self.ln_eps)
        self.packed = torch.empty(int(self._lib.dd_mlp_packed_floats()), dtype=torch.float32, device=self.device)
        abi.check(self._lib.dd_mlp_pack(ctypes.byref(p), self._mode, self.packed.data_ptr(), self._stream()),
                  "dd_mlp_pack")

    @classmethod
    def from_file(cls, path: str, **kw) -> "MlpNet":
        """Load a notebook checkpoint (a state_dict) without unpickling code."""
        return cls(torch.load(path, map_location="cpu", weights_only=True), **kw)

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _obs(self, obs: torch.Tensor) -> torch.Tensor:
        if obs.dim() != 2 or obs.shape[1] != abi.DD_OBS_DIM:
            raise ValueError(f"obs must be [N, {abi.DD_OBS_DIM}], got {tuple(obs.shape)}")
        if obs.device != self.device:
            raise ValueError(f"obs is on {obs.device}, the network on {self.device}")
        return obs.to(torch.float32).contiguous()

    def _run(self, obs, out=None, actions=None, log_prob=None, seed=0, step=0, env_id_base=0):
        io = abi.DDMlpIO(obs.data_ptr(), out.data_ptr() if out is not None else None,
                         actions.data_ptr() if actions is not None else None,
                         log_prob.data_ptr() if log_prob is not None else None,
                         int(seed) & (2 ** 64 - 1), int(step), int(env_id_base))
        abi.check(self._lib.dd_mlp_forward(self.packed.data_ptr(), self._mode, self.out_dim, ctypes.byref(io),
                                           obs.shape[0], self._stream()), "dd_mlp_forward")

    def __call__(self, obs: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``network(obs)``: probabilities ``[N, 3]`` (actor) or values ``[N]`` (critic)."""
        obs = self._obs(obs)
        n = obs.shape[0]
        if out is None:
            out = torch.empty((n, 3) if self.out_dim == 3 else (n,), dtype=torch.float32, device=self.device)
        self._run(obs, out=out)
        return out

    def act(self, obs: torch.Tensor, *, seed: int = 0, step: int = 0, env_id_base: int = 0,
            probs: bool = False, actions_out: Optional[torch.Tensor] = None,
            log_prob_out: Optional[torch.Tensor] = None):
        """Sample actions as the collection loop does (actor only).

        Returns ``(actions, log_prob)`` or ``(actions, log_prob, probs)``:
        actions is the uint8 ``[N]`` bitmask ``dd_step`` consumes (bit 0 main,
        1 left, 2 right), log_prob the float32 ``[N]`` sum over the three
        Bernoulli factors.  Draws are Philox4x32-10 keyed by (seed; env id,
        step), so a lane's sample does not depend on sharding.
        """
        if self.out_dim != 3:
            raise ValueError("act() needs the actor (out_dim 3)")
        obs = self._obs(obs)
        n = obs.shape[0]
        actions = actions_out if actions_out is not None else torch.empty(n, dtype=torch.uint8, device=self.device)
        log_prob = log_prob_out if log_prob_out is not None else torch.empty(n, dtype=torch.float32,
                                                                             device=self.device)
        p = torch.empty(n, 3, dtype=torch.float32, device=self.device) if probs else None
        self._run(obs, out=p, actions=actions, log_prob=log_prob, seed=seed, step=step, env_id_base=env_id_base)
        return (actions, log_prob, p) if probs else (actions, log_prob)
