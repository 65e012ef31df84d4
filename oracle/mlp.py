"""tiny-cuda-nn v1.7 ``FullyFusedMLP`` restated in numpy — TEST INFRASTRUCTURE ONLY.

Reference call sites: ``src/models/nerf_tcnn.py:35-38`` (sigma net: 32 -> 64 ReLU -> 1, config
``cfg/nerf_config/default_nerf_hash.yaml:26-31``) and ``:50-52`` (RGB net: 48 -> 4x64 -> 3).
tcnn semantics (unpinned, tcnn is not vendored): no biases, ReLU hidden activations,
``output_activation: None``, output width padded to 16, fp16 weights and activations.
The build (and this oracle) accumulates in fp32, rounds hidden activations to fp16 before the
next layer and rounds the network output to fp16 (tcnn returns fp16).

Weight layout used by the build (tcnn's internal layout cannot be observed here): one row-major
``[out][in]`` matrix per layer, concatenated first layer -> last layer.
"""
import numpy as np


def splitmix64(x):
    x = (np.asarray(x, dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15))
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def uniform_fill(n, seed, lo, hi, start=0):
    """Counter-based U(lo, hi) fill, identical to ``lnr_fill_uniform`` in the C-ABI."""
    with np.errstate(over="ignore"):
        i = np.arange(start, start + n, dtype=np.uint64)
        u = (splitmix64(i + (np.uint64(seed) << np.uint64(32))) >> np.uint64(40)).astype(np.float64) * 2.0 ** -24
    return (np.float32(lo) + np.float32(hi - lo) * u.astype(np.float32)).astype(np.float32)


def layer_shapes(n_input, n_output, width=64, n_hidden_layers=1):
    """[(out, in)] per weight matrix; output padded to a multiple of 16 (tcnn)."""
    pad_out = ((n_output + 15) // 16) * 16
    pad_in = ((n_input + 15) // 16) * 16
    shapes = [(width, pad_in)]
    shapes += [(width, width)] * (n_hidden_layers - 1)
    shapes.append((pad_out, width))
    return shapes


def unflatten(params, shapes):
    mats, off = [], 0
    for (o, i) in shapes:
        mats.append(np.asarray(params[off:off + o * i]).reshape(o, i))
        off += o * i
    return mats


def forward(x_f16, mats_f16):
    """x (N, in) fp16, mats [(out,in)] fp16 -> (out (N, pad_out) fp16, hidden list fp16)."""
    h = np.asarray(x_f16).astype(np.float32)
    hidden = []
    for li, w in enumerate(mats_f16):
        a = h.astype(np.float64) @ np.asarray(w).astype(np.float64).T
        if li < len(mats_f16) - 1:
            a = np.maximum(a, 0.0)
            h = a.astype(np.float32).astype(np.float16)
            hidden.append(h)
            h = h.astype(np.float32)
        else:
            return a.astype(np.float32).astype(np.float16), hidden
    raise AssertionError("unreachable")


def backward(x_f16, mats_f16, hidden, d_out):
    """d_out (N, pad_out) fp32/64 -> (d_x (N, in) fp64, [dW (out,in) fp64])."""
    acts = [np.asarray(x_f16).astype(np.float64)] + [np.asarray(h).astype(np.float64) for h in hidden]
    g = np.asarray(d_out, dtype=np.float64)
    dws = [None] * len(mats_f16)
    for li in range(len(mats_f16) - 1, -1, -1):
        w = np.asarray(mats_f16[li]).astype(np.float64)
        dws[li] = g.T @ acts[li]
        g = g @ w
        if li > 0:
            g = g * (acts[li] > 0)
    return g, dws
