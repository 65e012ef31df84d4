"""tiny-cuda-nn v1.7 ``HashGrid`` restated in numpy — TEST INFRASTRUCTURE ONLY.

Reference call site: ``src/models/nerf_tcnn.py:35-38`` (sigma head) and ``:42`` (RGB head), config
``cfg/nerf_config/default_nerf_hash.yaml:14-25`` (L=16, F=2, log2 T=18/19, N_min=16,
per_level_scale unset -> tcnn default 2.0).  tcnn is not vendored in ``/root/reference`` and is
CUDA-only, so this restatement follows tcnn v1.7's published algorithm (``grid.h``:
``grid_scale``, ``grid_resolution``, ``grid_index``, ``coherent_prime_hash``, ``kernel_grid``,
``kernel_grid_backward``) and is **parity unpinned** against tcnn itself.

Emulation choices shared with the HIP kernels (documented in DESIGN.md):
  * table values are fp16 (tcnn forwards with fp16 params); interpolation weights and the
    8-corner accumulation are fp32 (tcnn: fp16 ``fma``); the encoding is rounded to fp16 once;
  * backward accumulates fp32 gradients (tcnn: fp16 atomics under loss scale 128).
"""
import numpy as np

PRIMES = (np.uint64(1), np.uint64(2654435761), np.uint64(805459861))
_M = np.uint64(0xFFFFFFFF)


class GridLayout:
    """Per-level scale / resolution / size / offset (tcnn ``GridEncodingTemplated`` ctor)."""

    def __init__(self, n_levels=16, n_features=2, log2_hashmap_size=18, base_resolution=16,
                 per_level_scale=2.0):
        self.n_levels = n_levels
        self.n_features = n_features
        self.log2_hashmap_size = log2_hashmap_size
        self.base_resolution = base_resolution
        self.per_level_scale = per_level_scale
        l2s = np.float32(np.log2(np.float32(per_level_scale)))
        self.scales, self.resolutions, self.sizes, self.offsets = [], [], [], []
        offset = 0
        max_params = (2 ** 32 - 1) // 2
        for lvl in range(n_levels):
            scale = np.float32(np.float32(np.exp2(np.float32(lvl) * l2s)) * np.float32(base_resolution)) - np.float32(1.0)
            res = int(np.ceil(scale)) + 1
            dense = res ** 3 if float(res) ** 3 <= float(max_params) else max_params
            size = ((dense + 7) // 8) * 8
            size = min(size, 1 << log2_hashmap_size)
            self.scales.append(np.float32(scale))
            self.resolutions.append(res)
            self.sizes.append(size)
            self.offsets.append(offset)
            offset += size
        self.n_entries = offset
        self.n_params = offset * n_features
        self.n_output_dims = n_levels * n_features


def grid_index(cell, res, size):
    """tcnn ``grid_index`` for 3-D HashGrid: dense stride walk, prime hash once stride > size."""
    cell = cell.astype(np.uint64)
    stride = 1
    index = np.zeros(cell.shape[:-1], dtype=np.uint64)
    for d in range(3):
        if stride > size:
            break
        index = (index + cell[..., d] * np.uint64(stride)) & _M
        stride *= res
    if size < stride:
        h = np.zeros_like(index)
        for d in range(3):
            h ^= (cell[..., d] * PRIMES[d]) & _M
        index = h
    return (index % np.uint64(size)).astype(np.int64)


def _corners(pos01, layout, lvl):
    """fp32 grid position, integer cell and fraction for one level (tcnn ``pos_fract``)."""
    scale = layout.scales[lvl]
    p = (np.float64(scale) * pos01.astype(np.float64) + 0.5).astype(np.float32)  # fmaf(scale, x, 0.5)
    fl = np.floor(p)
    return fl.astype(np.int64), (p - fl).astype(np.float32)


def corner_weights_indices(pos01, layout, lvl):
    """(N, 8) fp32 trilinear weights and (N, 8) global entry indices, corner order idx=0..7
    with bit d selecting +1 along dimension d (tcnn ``kernel_grid`` loop order)."""
    cell, frac = _corners(pos01, layout, lvl)
    one = np.float32(1.0)
    ws, ids = [], []
    for c in range(8):
        w = np.ones(pos01.shape[0], dtype=np.float32)
        cc = cell.copy()
        for d in range(3):
            if (c >> d) & 1:
                w = (w * frac[:, d]).astype(np.float32)
                cc[:, d] += 1
            else:
                w = (w * (one - frac[:, d])).astype(np.float32)
        ws.append(w)
        ids.append(layout.offsets[lvl] + grid_index(cc, layout.resolutions[lvl], layout.sizes[lvl]))
    return np.stack(ws, 1), np.stack(ids, 1)


def encode(pos01, table_f16, layout):
    """Forward: pos01 (N,3) fp32 in [0,1]^3, table (n_entries, F) fp16 -> (N, L*F) fp16.
    Output order is level-major [l0f0, l0f1, l1f0, ...] (tcnn AoS output)."""
    pos01 = np.asarray(pos01, dtype=np.float32)
    tab = np.asarray(table_f16).astype(np.float32)
    n = pos01.shape[0]
    out = np.zeros((n, layout.n_output_dims), dtype=np.float32)
    for lvl in range(layout.n_levels):
        w, idx = corner_weights_indices(pos01, layout, lvl)
        acc = np.zeros((n, layout.n_features), dtype=np.float32)
        for c in range(8):
            acc = (acc + w[:, c:c + 1] * tab[idx[:, c]]).astype(np.float32)
        out[:, lvl * layout.n_features:(lvl + 1) * layout.n_features] = acc
    return out.astype(np.float16)


def encode_input_grad(pos01, table_f16, d_enc, layout, exact=False):
    """Input gradient: d_enc (N, L*F) -> dL/dpos01 (N, 3) fp64.  tcnn v1.7 ``grid.h``: ``kernel_grid``
    with ``dy_dx`` (per level, feature and axis: over the 4 cell edges along the axis, scale_l times
    the product of the other axes' weights times (upper corner value - lower corner value), the other
    axes in increasing order; ``pos_derivative`` = 1 for linear interpolation) and
    ``kernel_grid_backward_input`` (dL/dx = sum over output features of dL/dy * dy/dx).  Table values
    are the fp16 forward operand, cell fractions fp32 as in the forward (tcnn: fmaf(scale, x, 0.5f)); the
    sums are fp64 here.  ``exact``: fractions from fp64 positions instead (the derivative of
    ``encode_f64``, for the central-difference check of the formula itself)."""
    pos64 = np.asarray(pos01, dtype=np.float64)
    pos01 = np.asarray(pos01, dtype=np.float32)
    tab = np.asarray(table_f16).astype(np.float64)
    d_enc = np.asarray(d_enc, dtype=np.float64)
    n = pos01.shape[0]
    out = np.zeros((n, 3), dtype=np.float64)
    for lvl in range(layout.n_levels):
        if exact:
            pf = pos64 * np.float64(layout.scales[lvl]) + 0.5
            cell = np.floor(pf).astype(np.int64)
            frac = pf - cell
        else:
            cell, frac = _corners(pos01, layout, lvl)
            frac = frac.astype(np.float64)
        scale = np.float64(layout.scales[lvl])
        res, size, off = layout.resolutions[lvl], layout.sizes[lvl], layout.offsets[lvl]
        dl = d_enc[:, lvl * layout.n_features:(lvl + 1) * layout.n_features]
        for dim in range(3):
            others = [d for d in range(3) if d != dim]
            acc = np.zeros((n, layout.n_features))
            for e in range(4):
                w = np.full(n, scale)
                lo = cell.copy()
                for j, od in enumerate(others):
                    bit = (e >> j) & 1
                    w = w * (frac[:, od] if bit else 1.0 - frac[:, od])
                    lo[:, od] += bit
                hi = lo.copy()
                hi[:, dim] += 1
                v_lo = tab[off + grid_index(lo, res, size)]
                v_hi = tab[off + grid_index(hi, res, size)]
                acc += w[:, None] * (v_hi - v_lo)
            out[:, dim] += (dl * acc).sum(-1)
    return out


def encode_f64(pos01, table, layout):
    """The trilinear blend in fp64 throughout (no fp32 fractions, no fp16 output rounding): the smooth
    function whose central differences check ``encode_input_grad`` (tests/test_oracle_tcnn.py)."""
    pos01 = np.asarray(pos01, dtype=np.float64)
    tab = np.asarray(table).astype(np.float64)
    out = np.zeros((pos01.shape[0], layout.n_output_dims))
    for lvl in range(layout.n_levels):
        p = pos01 * np.float64(layout.scales[lvl]) + 0.5
        cell = np.floor(p).astype(np.int64)
        frac = p - cell
        acc = np.zeros((pos01.shape[0], layout.n_features))
        for c in range(8):
            w = np.ones(pos01.shape[0])
            cc = cell.copy()
            for d in range(3):
                if (c >> d) & 1:
                    w = w * frac[:, d]
                    cc[:, d] += 1
                else:
                    w = w * (1.0 - frac[:, d])
            acc += w[:, None] * tab[layout.offsets[lvl] + grid_index(cc, layout.resolutions[lvl], layout.sizes[lvl])]
        out[:, lvl * layout.n_features:(lvl + 1) * layout.n_features] = acc
    return out


def encode_backward(pos01, d_enc, layout):
    """Backward: d_enc (N, L*F) -> dtable (n_entries, F) fp64 (scatter-add of w * d_enc)."""
    pos01 = np.asarray(pos01, dtype=np.float32)
    d_enc = np.asarray(d_enc, dtype=np.float64)
    g = np.zeros((layout.n_entries, layout.n_features), dtype=np.float64)
    for lvl in range(layout.n_levels):
        w, idx = corner_weights_indices(pos01, layout, lvl)
        dl = d_enc[:, lvl * layout.n_features:(lvl + 1) * layout.n_features]
        for c in range(8):
            np.add.at(g, idx[:, c], w[:, c:c + 1].astype(np.float64) * dl)
    return g
