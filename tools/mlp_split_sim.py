#!/usr/bin/env python
"""numpy emulation of the DD_MLP_F16X3 split-operand GEMMs on the notebook models
(tests/golden/policy.npz): max probability / value error against float64, next
to plain float32.  Operands split as a = hi + lo * 2^-11 with hi, lo f16
(both rounded to nearest-even: truncating them, v_cvt_pkrtz, biases lo and
quadruples the error; run with --truncate), products exact, sums rounded to f32.
--center: the hidden Linears mean-centred over their outputs and the LayerNorm
without its mean pass, as dd_mlp_pack / norm_relu_emit do (mlp_core.h kCentered).
The `single` rows emulate the round-5 form (mlp_core.h): lo = f16(a - hi)
unscaled, the three products in one accumulator from the bias, hidden weights
x16, the layer-1 input x64, LayerNorm outputs x16 (powers of two the
LayerNorms remove), centred weights.  The `rtz` rows (the kernels since late
round 5): the LayerNorm outputs split with their ReLU (mlp_core.h
split_pair_relu: hi rounded toward zero and raised to 0, lo = RNE of the
clamped residual).  The `clamp` rows (tried and dropped): every LayerNorm's
output scaled by the per-layer power of two that keeps it below 1, so that
ReLU is the FMA's clamp modifier; lo then often sits in the f16 subnormals."""
import sys

import numpy as np

TRUNCATE = '--truncate' in sys.argv
CENTER = '--center' in sys.argv
d = np.load(__import__('os').path.join(__import__('os').path.dirname(__import__('os').path.abspath(__file__)), '..', 'tests', 'golden', 'policy.npz'))
def rtz16(x):
    """float32 -> float16 rounded toward zero (v_cvt_pkrtz_f16_f32)."""
    h = x.astype(np.float16)
    over = np.abs(h.astype(np.float32)) > np.abs(x)
    return np.where(over, np.nextafter(h, np.float16(0)), h)


def split(a):
    a = a.astype(np.float32)
    hi = a.astype(np.float16)  # v_cvt_pk_f16_f32, nearest-even; a - hi is exact
    lo = ((a - hi.astype(np.float32)) * np.float32(2048)).astype(np.float16)
    if TRUNCATE:  # the v_cvt_pkrtz_f16_f32 form, for comparison
        hi = rtz16(a)
        lo = rtz16((a - hi.astype(np.float32)) * np.float32(2048))
    return hi, lo
def lin(W, x, b, mode):
    # W [o,i], x [n,i]
    if mode == 'f64':
        return x.astype(np.float64) @ W.T.astype(np.float64) + b
    if mode == 'f32':
        return (x.astype(np.float32) @ W.T.astype(np.float32) + b).astype(np.float32)
    Wh, Wl = split(W); xh, xl = split(x)
    f = lambda a: a.astype(np.float64)
    main = f(xh) @ f(Wh).T
    cross = (f(xh) @ f(Wl).T + f(xl) @ f(Wh).T)
    # emulate f32 accumulation coarsely: round each sum to f32
    return (main.astype(np.float32) + (cross.astype(np.float32) * np.float32(2**-11))).astype(np.float32) + b
def ln(x, w, b, mode):
    dt = np.float64 if mode == 'f64' else np.float32
    x = x.astype(dt); m = x.mean(1, keepdims=True)
    if CENTER and mode != 'f64':
        m = np.zeros_like(m)  # the centred GEMM's output: mean zero to rounding
    v = ((x - m) ** 2).mean(1, keepdims=True)
    return np.maximum((x - m) / np.sqrt(v + 1e-5) * w + b, 0)
def fwd(pre, mode):
    x = d['obs']
    for i, j in ((0, 1), (3, 4), (6, 7)):
        W, b = d[f'{pre}.network.{i}.weight'], d[f'{pre}.network.{i}.bias']
        if CENTER and mode != 'f64':
            W = (W.astype(np.float64) - W.astype(np.float64).mean(0, keepdims=True)).astype(np.float32)
            b = (b.astype(np.float64) - b.astype(np.float64).mean()).astype(np.float32)
        x = lin(W, x, b, mode)
        x = ln(x, d[f'{pre}.network.{j}.weight'], d[f'{pre}.network.{j}.bias'], mode)
    z = lin(d[f'{pre}.network.9.weight'], x, d[f'{pre}.network.9.bias'], 'f64' if mode == 'f64' else 'f32')
    return z
for pre in ('actor', 'critic'):
    ref = fwd(pre, 'f64')
    for mode in ('f32', 'split'):
        z = fwd(pre, mode)
        if pre == 'actor':
            p = 1/(1+np.exp(-z.astype(np.float64))); pr = 1/(1+np.exp(-ref))
            print(pre, mode, 'max |dprob| vs f64', np.abs(p - pr).max(), 'vs golden', np.abs(p - d['probs']).max())
        else:
            print(pre, mode, 'max |dv| vs f64', np.abs(z[:,0]-ref[:,0]).max(), 'vs golden', np.abs(z[:,0]-d['values']).max(), 'max|v|', np.abs(ref).max())


def split_unscaled(a):
    a = a.astype(np.float32)
    hi = a.astype(np.float16)
    return hi, (a - hi.astype(np.float32)).astype(np.float16)  # lo may be an f16 subnormal


def fwd_single(pre, w=4, am=4, im=6):
    """The round-5 f16x3 form; the power-of-two scales of mlp_core.h (kWScale 2^w,
    kInScale 2^im, LayerNorm outputs x 2^am)."""
    f = lambda a: a.astype(np.float64)  # noqa: E731
    x = d['obs'].astype(np.float32) * np.float32(2.0 ** im)
    s_in = 2.0 ** im
    for i, j in ((0, 1), (3, 4), (6, 7)):
        W, b = d[f'{pre}.network.{i}.weight'], d[f'{pre}.network.{i}.bias']
        W = (W.astype(np.float64) - W.astype(np.float64).mean(0, keepdims=True)).astype(np.float32)
        b = (b.astype(np.float64) - b.astype(np.float64).mean()).astype(np.float32)
        Wh, Wl = split_unscaled(W * np.float32(2.0 ** w))
        xh, xl = split_unscaled(x)
        sc = np.float32(2.0 ** w * s_in)
        acc = (f(xh) @ f(Wh).T + f(xh) @ f(Wl).T + f(xl) @ f(Wh).T + f((b * sc).astype(np.float32))).astype(np.float32)
        z = acc * (1 / np.sqrt((acc ** 2).mean(1, keepdims=True) + np.float32(1e-5) * sc * sc))
        g = d[f'{pre}.network.{j}.weight'].astype(np.float32) * np.float32(2.0 ** am)
        be = d[f'{pre}.network.{j}.bias'].astype(np.float32) * np.float32(2.0 ** am)
        x = np.maximum(z * g + be, 0).astype(np.float32)
        s_in = 2.0 ** am
    W4 = d[f'{pre}.network.9.weight'].astype(np.float32) * np.float32(2.0 ** -am)
    return (x @ W4.T + d[f'{pre}.network.9.bias']).astype(np.float32)


for pre in ('actor', 'critic'):
    ref = fwd(pre, 'f64')
    z = fwd_single(pre)
    if pre == 'actor':
        p = 1 / (1 + np.exp(-z.astype(np.float64)))
        print(pre, 'single', 'max |dprob| vs f64', np.abs(p - 1 / (1 + np.exp(-ref))).max())
    else:
        print(pre, 'single', 'max |dv| vs f64', np.abs(z[:, 0] - ref[:, 0]).max())


def act_scale(pre, j, rows):
    """policy_mlp.hip act_scale: 2^-x with max|g| sqrt(rows) (1 + 2^-8) + max|b| = m 2^x, m in [0.5, 1)."""
    g = np.abs(d[f'{pre}.network.{j}.weight']).max()
    b = np.abs(d[f'{pre}.network.{j}.bias']).max()
    bound = np.float32(g) * np.float32(np.sqrt(rows)) * np.float32(1 + 2.0 ** -8) + np.float32(b)
    return 1.0 if not bound > 0 else float(2.0 ** -np.frexp(bound)[1])


def fwd_clamp(pre, w=4, im=6):
    """The clamp form: fwd_single with per-layer activation scales below 1."""
    f = lambda a: a.astype(np.float64)  # noqa: E731
    x = d['obs'].astype(np.float32) * np.float32(2.0 ** im)
    s_in = 2.0 ** im
    for (i, j), rows in zip(((0, 1), (3, 4), (6, 7)), (128, 128, 64)):
        W, b = d[f'{pre}.network.{i}.weight'], d[f'{pre}.network.{i}.bias']
        W = (W.astype(np.float64) - W.astype(np.float64).mean(0, keepdims=True)).astype(np.float32)
        b = (b.astype(np.float64) - b.astype(np.float64).mean()).astype(np.float32)
        Wh, Wl = split_unscaled(W * np.float32(2.0 ** w))
        xh, xl = split_unscaled(x)
        sc = np.float32(2.0 ** w * s_in)
        acc = (f(xh) @ f(Wh).T + f(xh) @ f(Wl).T + f(xl) @ f(Wh).T + f((b * sc).astype(np.float32))).astype(np.float32)
        z = acc * (1 / np.sqrt((acc ** 2).mean(1, keepdims=True) + np.float32(1e-5) * sc * sc))
        s_out = act_scale(pre, j, rows)
        g = d[f'{pre}.network.{j}.weight'].astype(np.float32) * np.float32(s_out)
        be = d[f'{pre}.network.{j}.bias'].astype(np.float32) * np.float32(s_out)
        v = (z * g + be).astype(np.float32)
        assert v.max() < 1.0
        x = np.clip(v, 0, 1).astype(np.float32)
        s_in = s_out
    W4 = d[f'{pre}.network.9.weight'].astype(np.float32) * np.float32(1.0 / s_in)
    return (x @ W4.T + d[f'{pre}.network.9.bias']).astype(np.float32)


for pre in ('actor', 'critic'):
    ref = fwd(pre, 'f64')
    z = fwd_clamp(pre)
    if pre == 'actor':
        p = 1 / (1 + np.exp(-z.astype(np.float64)))
        print(pre, 'clamp', 'max |dprob| vs f64', np.abs(p - 1 / (1 + np.exp(-ref))).max())
    else:
        print(pre, 'clamp', 'max |dv| vs f64', np.abs(z[:, 0] - ref[:, 0]).max())


def rtz16(x):
    h = x.astype(np.float16)
    over = np.abs(h.astype(np.float32)) > np.abs(x)
    return np.where(over, np.nextafter(h, np.float16(0)), h)


def split_relu(a):
    """split_pair_relu: hi = max(rtz16(a), 0), lo = f16(clamp(a - hi, 0, 1)) (RNE)."""
    a = a.astype(np.float32)
    hi = np.maximum(rtz16(a), np.float16(0))
    return hi, np.clip(a - hi.astype(np.float32), 0, 1).astype(np.float16)


def fwd_rtz(pre, w=4, am=4, im=6):
    """fwd_single with the hidden activations split by split_relu (ReLU inside the split)."""
    f = lambda a: a.astype(np.float64)  # noqa: E731
    x = d['obs'].astype(np.float32) * np.float32(2.0 ** im)
    s_in = 2.0 ** im
    for n, (i, j) in enumerate(((0, 1), (3, 4), (6, 7))):
        W, b = d[f'{pre}.network.{i}.weight'], d[f'{pre}.network.{i}.bias']
        W = (W.astype(np.float64) - W.astype(np.float64).mean(0, keepdims=True)).astype(np.float32)
        b = (b.astype(np.float64) - b.astype(np.float64).mean()).astype(np.float32)
        Wh, Wl = split_unscaled(W * np.float32(2.0 ** w))
        xh, xl = split_unscaled(x) if n == 0 else split_relu(x)
        sc = np.float32(2.0 ** w * s_in)
        acc = (f(xh) @ f(Wh).T + f(xh) @ f(Wl).T + f(xl) @ f(Wh).T + f((b * sc).astype(np.float32))).astype(np.float32)
        z = acc * (1 / np.sqrt((acc ** 2).mean(1, keepdims=True) + np.float32(1e-5) * sc * sc))
        g = d[f'{pre}.network.{j}.weight'].astype(np.float32) * np.float32(2.0 ** am)
        be = d[f'{pre}.network.{j}.bias'].astype(np.float32) * np.float32(2.0 ** am)
        x = (z * g + be).astype(np.float32)  # ReLU in the next split (or below, for the head)
        s_in = 2.0 ** am
    x = np.maximum(x, 0)
    W4 = d[f'{pre}.network.9.weight'].astype(np.float32) * np.float32(2.0 ** -am)
    return (x @ W4.T + d[f'{pre}.network.9.bias']).astype(np.float32)


for pre in ('actor', 'critic'):
    ref = fwd(pre, 'f64')
    z = fwd_rtz(pre)
    if pre == 'actor':
        p = 1 / (1 + np.exp(-z.astype(np.float64)))
        print(pre, 'rtz', 'max |dprob| vs f64', np.abs(p - 1 / (1 + np.exp(-ref))).max())
    else:
        print(pre, 'rtz', 'max |dv| vs f64', np.abs(z[:, 0] - ref[:, 0]).max())
