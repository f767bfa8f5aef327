#!/usr/bin/env python
"""numpy emulation: f16x3 accuracy of three ReLU forms against float64 on
networks whose LayerNorm weights spread over a range (random torch init,
weights logspace(lo, hi) shuffled, biases U(-0.2, 0.2)), and on the notebook
models (tests/golden/policy.npz):

  old    activations x16, ReLU by max(), RNE hi/lo split (mlp_core.h before)
  clamp  outputs scaled below 1 per layer (max|g| sqrt(rows) + max|b|), ReLU
         as the FMA's clamp: lo in the f16 subnormals (tried, dropped)
  rtz    activations x16, hi = max(rtz16(x), 0), lo = RNE16(clamp(x - hi))
         (split_pair_relu, the kernels' form)

    python tools/lab/mlp_relu_forms_sim.py
"""
import os
import sys

import numpy as np
import torch
from torch import nn

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rtz16(x):
    h = x.astype(np.float16)
    over = np.abs(h.astype(np.float32)) > np.abs(x)
    return np.where(over, np.nextafter(h, np.float16(0)), h)


def split(a):
    a = a.astype(np.float32)
    hi = a.astype(np.float16)
    return hi, (a - hi.astype(np.float32)).astype(np.float16)


def split_relu(a):
    a = a.astype(np.float32)
    hi = np.maximum(rtz16(a), np.float16(0))
    return hi, np.clip(a - hi.astype(np.float32), 0, 1).astype(np.float16)


def forward(sd, obs, mode):
    f = lambda a: a.astype(np.float64)  # noqa: E731
    x = obs.astype(np.float32) * np.float32(64)
    s_in = 64.0
    for n, ((i, j), rows) in enumerate(zip(((0, 1), (3, 4), (6, 7)), (128, 128, 64))):
        W = sd[f"{i}.weight"].astype(np.float64)
        W = (W - W.mean(0, keepdims=True)).astype(np.float32)
        b = sd[f"{i}.bias"].astype(np.float64)
        b = (b - b.mean()).astype(np.float32)
        Wh, Wl = split(W * np.float32(16))
        xh, xl = split_relu(x) if (mode == "rtz" and n > 0) else split(x)
        sc = np.float32(16 * s_in)
        acc = (f(xh) @ f(Wh).T + f(xh) @ f(Wl).T + f(xl) @ f(Wh).T + f((b * sc).astype(np.float32))).astype(np.float32)
        z = acc * (1 / np.sqrt((acc ** 2).mean(1, keepdims=True) + np.float32(1e-5) * sc * sc))
        g_, b_ = sd[f"{j}.weight"], sd[f"{j}.bias"]
        if mode == "clamp":
            bound = np.float32(np.abs(g_).max()) * np.float32(np.sqrt(rows)) * np.float32(1 + 2.0 ** -8) \
                + np.float32(np.abs(b_).max())
            so = 1.0 if not bound > 0 else float(2.0 ** -np.frexp(bound)[1])
        else:
            so = 16.0
        v = (z * (g_ * np.float32(so)) + b_ * np.float32(so)).astype(np.float32)
        x = v if mode == "rtz" else np.maximum(v, 0).astype(np.float32)
        s_in = so
    x = np.maximum(x, 0)
    return (x @ (sd["9.weight"] * np.float32(1 / s_in)).T + sd["9.bias"]).astype(np.float64)


def reference(sd, obs):
    x = obs.astype(np.float64)
    for i, j in ((0, 1), (3, 4), (6, 7)):
        x = x @ sd[f"{i}.weight"].T.astype(np.float64) + sd[f"{i}.bias"]
        m = x.mean(1, keepdims=True)
        v = ((x - m) ** 2).mean(1, keepdims=True)
        x = np.maximum((x - m) / np.sqrt(v + 1e-5) * sd[f"{j}.weight"] + sd[f"{j}.bias"], 0)
    return x @ sd["9.weight"].T.astype(np.float64) + sd["9.bias"]


def main():
    modes = ("old", "clamp", "rtz")
    d = np.load(os.path.join(REPO, "tests", "golden", "policy.npz"))
    for pre in ("actor", "critic"):
        sd = {k.split("network.")[1]: d[k] for k in d.files if k.startswith(pre + ".network.")}
        ref = reference(sd, d["obs"])
        errs = []
        for m in modes:
            out = forward(sd, d["obs"], m)
            e = np.abs(1 / (1 + np.exp(-out)) - 1 / (1 + np.exp(-ref))).max() if pre == "actor" \
                else np.abs(out[:, 0] - ref[:, 0]).max()
            errs.append(f"{m} {e:.2e}")
        print(f"notebook {pre}:", *errs, flush=True)
    for lo, hi in ((-1, 0.7), (-2, 1), (-3, 1.7)):
        torch.manual_seed(11)
        net = nn.Sequential(nn.Linear(15, 128), nn.LayerNorm(128), nn.ReLU(), nn.Linear(128, 128), nn.LayerNorm(128),
                            nn.ReLU(), nn.Linear(128, 64), nn.LayerNorm(64), nn.ReLU(), nn.Linear(64, 3))
        with torch.no_grad():
            for i in (1, 4, 7):
                w = torch.logspace(lo, hi, net[i].weight.numel())
                net[i].weight.copy_(w[torch.randperm(w.numel())])
                net[i].bias.uniform_(-0.2, 0.2)
        sd = {k: v.numpy().astype(np.float32) for k, v in net.state_dict().items()}
        obs = (np.random.RandomState(0).randn(4097, 15) * 2).astype(np.float32)
        pr = 1 / (1 + np.exp(-reference(sd, obs)))
        errs = [f"{m} {np.abs(1 / (1 + np.exp(-forward(sd, obs, m))) - pr).max():.2e}" for m in modes]
        with torch.no_grad():
            pt = torch.sigmoid(net(torch.as_tensor(obs))).double().numpy()
        print(f"LayerNorm weights 10^{lo}..10^{hi}, actor probabilities:", *errs,
              f"torch-f32 {np.abs(pt - pr).max():.2e}", flush=True)


if __name__ == "__main__":
    sys.exit(main())
