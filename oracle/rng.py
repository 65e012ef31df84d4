"""Counter-based RNG shared bit-exactly with the HIP kernels (``loner_amd/csrc/common.hpp``).

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

The reference draws its three random streams from torch's global generator:
  * stratified jitter  ``torch.rand``  (``src/models/ray_sampling.py:71-72``)
  * inverse-CDF draws  ``torch.rand``  (``src/models/rendering_tcnn.py:49``)
  * sigma noise        ``torch.randn`` (``src/models/rendering_tcnn.py:251-252``)
A GPU build cannot reproduce torch's Philox/MT19937 stream, so the build defines its own
counter-based generator keyed by (step key, stream, global ray index, sample index).  Parity
tests either inject the reference's recorded draws or regenerate these draws here.
"""
import numpy as np

STREAM_JITTER = 1
STREAM_PDF = 2
STREAM_NOISE = 3  # uses 3 (radius) and 4 (angle)

_M = np.uint64(0xFFFFFFFF)


def mix32(x):
    """lowbias32 finaliser on uint32 arrays (wrapping arithmetic)."""
    x = np.asarray(x, dtype=np.uint64) & _M
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & _M
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & _M
    x ^= x >> np.uint64(16)
    return x


def step_key(seed: int, step: int) -> int:
    """Per-step key; identical to ``lnr_step_key`` in the C-ABI."""
    return int(mix32(mix32(np.uint64(seed & 0xFFFFFFFF)) ^ np.uint64(step & 0xFFFFFFFF)))


def rand_u32(key, stream, a, b):
    a = np.asarray(a, dtype=np.uint64)
    b = np.asarray(b, dtype=np.uint64)
    h = mix32(np.uint64(key) ^ ((np.uint64(stream) * np.uint64(0x9E3779B9)) & _M))
    h = mix32(h ^ a)
    h = mix32(h ^ ((b * np.uint64(0x85EBCA6B) + np.uint64(0x632BE5AB)) & _M))
    return h


def uniform(key, stream, a, b):
    """U[0,1) with 24 random bits (same lattice as torch.rand for fp32)."""
    return ((rand_u32(key, stream, a, b) >> np.uint64(8)).astype(np.float64) * 2.0 ** -24).astype(np.float32)


def normal(key, stream, a, b):
    """Box-Muller N(0,1); radius from ``stream``, angle from ``stream + 1``."""
    u1 = ((rand_u32(key, stream, a, b) >> np.uint64(8)).astype(np.float64) + 1.0) * 2.0 ** -24
    u2 = (rand_u32(key, stream + 1, a, b) >> np.uint64(8)).astype(np.float64) * 2.0 ** -24
    return (np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)).astype(np.float32)


def ray_sample_grid(ray_ids, n):
    """(R, n) index grids (a = global ray id, b = sample id) for vectorised draws."""
    a = np.repeat(np.asarray(ray_ids, dtype=np.uint64)[:, None], n, axis=1)
    b = np.repeat(np.arange(n, dtype=np.uint64)[None, :], len(ray_ids), axis=0)
    return a, b
