"""Draw keys for the tcnn-compatible render path.

The reference draws its jitter, inverse-CDF and sigma-noise variates with ``torch.rand`` /
``torch.randn`` (ray_sampling.py:41,73; rendering_tcnn.py:252).  The HIP kernels instead use a
counter-based generator (loner_amd/csrc/common.hpp, oracle/rng.py) keyed by a 32-bit key and the
(ray, sample) index, so draws are reproducible across launches, batch splits and GPUs.  Each
sampler / render call takes the next key of a process-wide sequence seeded by ``manual_seed``.
"""
from . import _lib as L

_state = {"seed": 0, "counter": 0}


def manual_seed(seed: int) -> None:
    _state["seed"] = int(seed) & 0xFFFFFFFF
    _state["counter"] = 0


def next_key() -> int:
    k = L.step_key(_state["seed"], _state["counter"])
    _state["counter"] += 1
    return k
