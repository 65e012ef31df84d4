"""Parity of the HIP path (through the C ABI) against the CPU oracle and the reference's golden
vectors.  GPU only: run with ``pytest -m gpu`` on an MI355X.

Tolerances: integer/index work bit-exact (encoding indices, sorted sample
order); fp32 elementwise within a few ulp; fp16 outputs (encodings, sigma) within 1-2 fp16 ulp;
reductions/scans within 1e-5 relative; gradients of fp32 atomics within 1e-4 relative L2.
"""
import ast
import ctypes

import numpy as np
import pytest
import torch

from conftest import TABLE_GRAD_RTOL
from oracle import hashgrid as ohg
from oracle import loss as oloss
from oracle import mlp as omlp
from oracle import optim as ooptim
from oracle import render as orender
from oracle import rng as orng

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from loner_amd import _lib
    _lib.lib()
    return _lib


def cu(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def enc_levelmajor_to_aos(enc_i32, n, L_):
    e = host(enc_i32).view(np.uint32).reshape(L_, -1)[:, :n]
    lo = (e & 0xFFFF).astype(np.uint16).view(np.float16)
    hi = (e >> 16).astype(np.uint16).view(np.float16)
    out = np.empty((n, 2 * L_), np.float16)
    out[:, 0::2] = lo.T
    out[:, 1::2] = hi.T
    return out


# ------------------------------------------------------------------ hash grid
def test_hashgrid_fwd_bitexact_indices(L):
    rng = np.random.default_rng(0)
    n = 5000
    lay = ohg.GridLayout(16, 2, 18, 16)
    d = L.grid_desc(16, 2, 18, 16)
    pos = rng.uniform(0, 1, (n, 3)).astype(np.float32)
    pos[:5] = [[0, 0, 0], [1, 1, 1], [0.5, 0.5, 0.5], [1, 0, 1], [0.999999, 0.3, 0.0]]
    table = rng.uniform(-1, 1, (lay.n_entries, 2)).astype(np.float16)
    enc = torch.empty(16, n, dtype=torch.int32, device="cuda")
    L.call("lnr_hashgrid_fwd", ctypes.byref(d), (cu(pos)), n, (cu(table.view(np.uint16).view(np.int16))),
           (enc), n, None, 0, L.stream())
    got = enc_levelmajor_to_aos(enc, n, 16).astype(np.float32)
    ref = ohg.encode(pos, table, lay).astype(np.float32)
    # identical corner indices and weights; only fp32 fma-vs-mul/add rounding differs -> <= 1 fp16 ulp
    ulp = np.abs(ref) * 2.0 ** -10 + 2.0 ** -24
    assert np.all(np.abs(got - ref) <= 1.01 * ulp), np.abs(got - ref).max()


@pytest.mark.parametrize("count", [False, True])
@pytest.mark.parametrize("n", [3 * 4096 + 77, (1 << 18) + 77])
def test_hashgrid_fwd_table_offset_and_ragged_rows(L, count, n):
    """The encode (lane-paired fine gathers: both lanes of a pair read one sample's x-pair, then swap)
    on a ragged last row of odd length (the last sample's partner lane has no sample), with the table at a 16-B aligned and at an unaligned (4 B past) address: the same
    entries, so bit-identical encodings and training-launch record histograms, and both within one
    fp16 ulp of the oracle.  Positions at the grid's upper edge exercise the x-pair wrap."""
    rng = np.random.default_rng(7)
    d = L.grid_desc(16, 2, 18, 16)
    lay = ohg.GridLayout(16, 2, 18, 16)
    pos = rng.uniform(0, 1, (n, 3)).astype(np.float32)
    pos[:6] = [[0, 0, 0], [1, 1, 1], [0.999999, 0.5, 0.25], [1, 0, 1], [0.5, 0.999999, 0.999999], [0.25, 0.75, 1]]
    table = rng.uniform(-1, 1, (lay.n_entries, 2)).astype(np.float16).view(np.int16).reshape(-1)
    buf = torch.zeros(table.size + 8, dtype=torch.int16, device="cuda")
    aligned = buf[:table.size]
    shifted = buf[2:2 + table.size]  # 4 B past a 16-B boundary
    outs = []
    for t in (aligned, shifted):
        t.copy_(torch.from_numpy(table))
        enc = torch.empty(16, n, dtype=torch.int32, device="cuda")
        ws = nb = None
        if count:
            nb = int(L.lib().lnr_hashgrid_bwd_workspace_bytes(ctypes.byref(d), n))
            ws = torch.zeros(nb // 4 + 1, dtype=torch.int32, device="cuda")
        L.call("lnr_hashgrid_fwd", ctypes.byref(d), cu(pos), n, t, enc, n, ws, nb or 0, L.stream())
        torch.cuda.synchronize()
        outs.append((enc.clone(), None if ws is None else ws.clone()))
    assert torch.equal(outs[0][0], outs[1][0])
    if count:
        assert torch.equal(outs[0][1], outs[1][1])
    got = enc_levelmajor_to_aos(outs[0][0], n, 16).astype(np.float32)
    ref = ohg.encode(pos, table.view(np.float16).reshape(-1, 2), lay).astype(np.float32)
    assert np.all(np.abs(got - ref) <= 1.01 * (np.abs(ref) * 2.0 ** -10 + 2.0 ** -24))


@pytest.mark.parametrize("R,lpb", [(24, "1"), (520, "1"), (520, "2")])
def test_hashgrid_fwd_live_mask_matches_full_encode(L, R, lpb, monkeypatch):
    """The live-masked eval encode (plain gathers, dead samples issue none; two samples per thread
    from 2^18 samples, or with LONER_ENC_LIVE_LPB=2 one sample per thread over two strided levels per
    workgroup) equals the full encode (lane-paired gathers) on live samples and is 0 on dead ones whose
    16-sample tile holds a live sample, bit for bit: the same entries in the same corner order.  A tile
    with no live sample is left unwritten."""
    monkeypatch.setenv("LONER_ENC_LIVE_LPB", lpb)
    rng = np.random.default_rng(11)
    S = 512
    d = L.grid_desc(16, 2, 19, 16)
    lay = ohg.GridLayout(16, 2, 19, 16)
    o = rng.uniform(-0.5, 0.5, (R, 3))
    dr = rng.normal(0, 1, (R, 3))
    dr /= np.linalg.norm(dr, axis=1, keepdims=True)
    rays = np.zeros((R, 13), np.float32)
    rays[:, 0:3], rays[:, 3:6] = o, dr
    z = np.sort(rng.uniform(0.0, 0.45, (R, S)), 1).astype(np.float32)
    live = (rng.uniform(0, 1, (R, S)) < 0.3).astype(np.float32)
    live.reshape(-1, 16)[rng.uniform(0, 1, R * S // 16) < 0.3] = 0.0  # whole dead tiles too
    table = cu(rng.uniform(-1, 1, (lay.n_entries, 2)).astype(np.float16).view(np.int16))
    full = torch.empty(16, R * S, dtype=torch.int32, device="cuda")
    part = torch.full((16, R * S), -1, dtype=torch.int32, device="cuda")
    L.call("lnr_hashgrid_fwd_rays", ctypes.byref(d), cu(rays), cu(z), R, S, table, full, R * S, None, 0, L.stream())
    L.call("lnr_hashgrid_fwd_rays_live", ctypes.byref(d), cu(rays), cu(z), R, S, table, cu(live), part, R * S,
           L.stream())
    alive = live.reshape(-1) != 0
    tile_live = np.repeat(alive.reshape(-1, 16).any(axis=1), 16)
    mask = torch.from_numpy(alive.reshape(1, -1)).cuda()
    want = torch.where(mask, full, torch.zeros_like(full))
    want[:, torch.from_numpy(~tile_live).cuda()] = -1  # unwritten
    assert tile_live.sum() < alive.size  # (the case is exercised)
    assert torch.equal(part, want)


@pytest.mark.parametrize("grid,R,S", [((16, 2, 19, 16), 520, 512), ((6, 2, 19, 16), 61, 40)])
def test_live_counted_backward(L, grid, R, S):
    """lnr_hashgrid_fwd_rays_live_ws counts the live samples' records while it encodes, and
    lnr_hashgrid_bwd_rays_live (LNR_BWD_COUNTS_READY) scatters exactly those: the same table gradient, bit
    for bit, as the backward counting for itself (by the mask, or by d_enc != 0 with no mask), since here every
    dead sample's d_enc is 0 and every live one's is not.  The colour grid at 520 rays (the level-looped
    scatter at 128 chunks per level) and a 6-level grid with a dense level past the merged ones (res 64 at
    40 samples per ray: the per-(row, level) scatter's generic path); the gradient against the oracle."""
    rng = np.random.default_rng(23)
    d = L.grid_desc(*grid)
    lay = ohg.GridLayout(*grid)
    nl = grid[0]
    o = rng.uniform(-0.5, 0.5, (R, 3))
    dr = rng.normal(0, 1, (R, 3))
    dr /= np.linalg.norm(dr, axis=1, keepdims=True)
    rays = np.zeros((R, 13), np.float32)
    rays[:, 0:3], rays[:, 3:6] = o, dr
    z = np.sort(rng.uniform(0.0, 0.45, (R, S)), 1).astype(np.float32)
    n = R * S
    live = (rng.uniform(0, 1, (R, S)) < 0.4).astype(np.float32)
    denc = rng.normal(0, 1, (n, 2 * nl)).astype(np.float32) * live.reshape(-1, 1)
    denc_lm = cu(np.ascontiguousarray(denc.reshape(n, nl, 2).transpose(1, 0, 2)))
    table = cu(rng.uniform(-1, 1, (lay.n_entries, 2)).astype(np.float16).view(np.int16))
    nb = int(L.lib().lnr_hashgrid_bwd_workspace_bytes(ctypes.byref(d), n))
    grads = []
    for mode in ("fwd_counts", "own_count_live", "own_count_nonzero"):
        ws = torch.zeros(nb // 4 + 1, dtype=torch.int32, device="cuda")
        enc = torch.full((nl, n), -1, dtype=torch.int32, device="cuda")
        gt = torch.full((lay.n_entries * 2,), 7.0, dtype=torch.float32, device="cuda")
        if mode == "fwd_counts":
            L.call("lnr_hashgrid_fwd_rays_live_ws", ctypes.byref(d), cu(rays), cu(z), R, S, table, cu(live), enc, n,
                   ws, nb, L.stream())
            ref_enc = torch.full((nl, n), -1, dtype=torch.int32, device="cuda")
            L.call("lnr_hashgrid_fwd_rays_live", ctypes.byref(d), cu(rays), cu(z), R, S, table, cu(live), ref_enc, n,
                   L.stream())
            assert torch.equal(enc, ref_enc)  # the counting changes no encoding
            L.call("lnr_hashgrid_bwd_rays_live", ctypes.byref(d), cu(rays), cu(z), R, S, denc_lm, n, cu(live), gt, ws,
                   nb, L.BWD_COUNTS_READY, L.stream())
        elif mode == "own_count_live":
            L.call("lnr_hashgrid_bwd_rays_live", ctypes.byref(d), cu(rays), cu(z), R, S, denc_lm, n, cu(live), gt, ws,
                   nb, 0, L.stream())
        else:
            L.call("lnr_hashgrid_bwd_rays", ctypes.byref(d), cu(rays), cu(z), R, S, denc_lm, n, gt, None, None, ws, nb,
                   0, L.stream())
        torch.cuda.synchronize()
        grads.append(gt.clone())
    assert torch.equal(grads[0], grads[1])
    assert torch.equal(grads[0], grads[2])
    o32, d32 = rays[:, None, 0:3], rays[:, None, 3:6]  # the kernels' fp32 op order: (o + d z + 1) * 0.5
    pos = (((o32 + d32 * z[:, :, None]) + np.float32(1)) * np.float32(0.5)).reshape(-1, 3)
    ref = ohg.encode_backward(pos, denc, lay)
    got = host(grads[0]).reshape(-1, 2)
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < TABLE_GRAD_RTOL


@pytest.mark.parametrize("S", [512, 64, 40])
def test_hashgrid_fwd_train_eval_live_agree(L, S):
    """The training launch (with the record histogram) and the plain eval launch give the same encodings, and
    the live-masked launch those encodings on its live samples; 40 samples per ray puts rays and ragged rows
    across waves.  (Round 5's run-head gathers on the coherent levels, which this test also pinned, were
    removed in round 6: measured no faster)"""
    rng = np.random.default_rng(5)
    R = 37
    d = L.grid_desc(16, 2, 18, 16)
    lay = ohg.GridLayout(16, 2, 18, 16)
    o = rng.uniform(-0.5, 0.5, (R, 3))
    dr = rng.normal(0, 1, (R, 3))
    dr /= np.linalg.norm(dr, axis=1, keepdims=True)
    rays = np.zeros((R, 13), np.float32)
    rays[:, 0:3], rays[:, 3:6] = o, dr
    z = np.sort(rng.uniform(0.0, 0.45, (R, S)), 1).astype(np.float32)
    z[:, S // 2:] = np.sort(0.2 + rng.uniform(-0.01, 0.01, (R, S - S // 2)), 1)  # long runs near a surface
    z = np.sort(z, 1)
    live = cu((rng.uniform(0, 1, (R, S)) < 0.5).astype(np.float32))
    table = cu(rng.uniform(-1, 1, (lay.n_entries, 2)).astype(np.float16).view(np.int16))
    n = R * S
    nb = int(L.lib().lnr_hashgrid_bwd_workspace_bytes(ctypes.byref(d), n))
    ws = torch.zeros(nb // 4 + 1, dtype=torch.int32, device="cuda")
    e_train = torch.full((16, n), -1, dtype=torch.int32, device="cuda")
    e_eval = torch.full((16, n), -1, dtype=torch.int32, device="cuda")
    e_live = torch.full((16, n), -1, dtype=torch.int32, device="cuda")
    L.call("lnr_hashgrid_fwd_rays", ctypes.byref(d), cu(rays), cu(z), R, S, table, e_train, n, ws, nb, L.stream())
    L.call("lnr_hashgrid_fwd_rays", ctypes.byref(d), cu(rays), cu(z), R, S, table, e_eval, n, None, 0, L.stream())
    L.call("lnr_hashgrid_fwd_rays_live", ctypes.byref(d), cu(rays), cu(z), R, S, table, live, e_live, n, L.stream())
    torch.cuda.synchronize()
    assert torch.equal(e_train, e_eval)
    m = live.reshape(-1) != 0
    assert torch.equal(e_live[:, m], e_eval[:, m])


@pytest.mark.parametrize("R", [520, 2060])
@pytest.mark.parametrize("nl", [15, 14])
def test_hashgrid_fwd_level_groups_bitwise(L, nl, R):
    """From 512 histogram rows a 16-level grid encodes two levels per workgroup (y, y + 8), from 2048
    rows four (y, y + 4, y + 8, y + 12); a 14-level grid two (y, y + 7) and a 15-level grid one: the
    levels the grids share have bit for bit the same encodings and training-launch record histograms."""
    rng = np.random.default_rng(17)
    S = 512
    o = rng.uniform(-0.5, 0.5, (R, 3))
    dr = rng.normal(0, 1, (R, 3))
    dr /= np.linalg.norm(dr, axis=1, keepdims=True)
    rays = np.zeros((R, 13), np.float32)
    rays[:, 0:3], rays[:, 3:6] = o, dr
    z = np.sort(rng.uniform(0.0, 0.45, (R, S)), 1).astype(np.float32)
    n = R * S
    lay = ohg.GridLayout(16, 2, 18, 16)
    table = cu(rng.uniform(-1, 1, (lay.n_entries, 2)).astype(np.float16).view(np.int16))
    outs = {}
    for g in (16, nl):
        d = L.grid_desc(g, 2, 18, 16)
        nb = int(L.lib().lnr_hashgrid_bwd_workspace_bytes(ctypes.byref(d), n))
        ws = torch.zeros(nb // 4 + 1, dtype=torch.int32, device="cuda")
        e_train = torch.full((g, n), -1, dtype=torch.int32, device="cuda")
        e_eval = torch.full((g, n), -1, dtype=torch.int32, device="cuda")
        L.call("lnr_hashgrid_fwd_rays", ctypes.byref(d), cu(rays), cu(z), R, S, table, e_train, n, ws, nb, L.stream())
        L.call("lnr_hashgrid_fwd_rays", ctypes.byref(d), cu(rays), cu(z), R, S, table, e_eval, n, None, 0, L.stream())
        torch.cuda.synchronize()
        outs[g] = (e_train, e_eval, ws)
    assert torch.equal(outs[16][0][:nl], outs[nl][0])
    assert torch.equal(outs[16][1][:nl], outs[nl][1])
    assert torch.equal(outs[16][0], outs[16][1])
    # histogram rows of the shared levels: the workspace's level maxima (256 B) come first, then the rows
    n_sb = (n + 511) // 512
    words = sum((s + 4095) // 4096 for s in lay.sizes[:nl]) * n_sb
    assert torch.equal(outs[16][2][64:64 + words], outs[nl][2][64:64 + words])


def test_hashgrid_fwd_rays_matches_positions(L):
    g = np.load("tests/golden/samplers.npz")
    rays, z = g["rays"], g["z_ogm"]
    R, S = z.shape
    lay = ohg.GridLayout(16, 2, 19, 16)  # the RGB-head grid (T=2^19)
    d = L.grid_desc(16, 2, 19, 16)
    rng = np.random.default_rng(1)
    table = rng.uniform(-1, 1, (lay.n_entries, 2)).astype(np.float16)
    enc = torch.empty(16, R * S, dtype=torch.int32, device="cuda")
    L.call("lnr_hashgrid_fwd_rays", ctypes.byref(d), (cu(rays)), (cu(z)), R, S,
           (cu(table.view(np.int16))), (enc), R * S, None, 0, L.stream())
    xyz = (rays[:, None, 0:3] + rays[:, None, 3:6] * z[:, :, None]).astype(np.float32)
    pos = ((xyz + np.float32(1)) / np.float32(2)).astype(np.float32).reshape(-1, 3)
    ref = ohg.encode(pos, table, lay).astype(np.float32)
    got = enc_levelmajor_to_aos(enc, R * S, 16).astype(np.float32)
    ulp = np.abs(ref) * 2.0 ** -10 + 2.0 ** -24
    assert np.all(np.abs(got - ref) <= 1.01 * ulp)


@pytest.mark.parametrize("variant", ["bucketed", "bucketed_fwd_counts", "atomic", "bucketed_scattered",
                                     "bucketed_scattered_fwd_counts"])
def test_hashgrid_bwd(L, variant):
    rng = np.random.default_rng(2)
    # a few "rays" of sorted samples so the coarse-level run merge is exercised
    R, S = 40, 256
    o = rng.uniform(-0.5, 0.5, (R, 3))
    dr = rng.normal(0, 1, (R, 3))
    dr /= np.linalg.norm(dr, axis=1, keepdims=True)
    t = np.sort(rng.uniform(0.0, 0.4, (R, S)), 1)
    pos = (((o[:, None] + dr[:, None] * t[:, :, None]) + 1) / 2).reshape(-1, 3).astype(np.float32)
    n = R * S - 77  # ragged tail
    pos = pos[:n]
    if "scattered" in variant:
        # unsorted positions: no runs merge, coherent rows carry 8 records per sample, more than the
        # level-looped scatter stages, so every coherent (row, level) takes the overflow pass
        pos = rng.uniform(0.0, 1.0, (n, 3)).astype(np.float32)
        variant = variant.replace("_scattered", "")
    lay = ohg.GridLayout(16, 2, 18, 16)
    d = L.grid_desc(16, 2, 18, 16)
    denc = rng.normal(0, 1, (n, 32)).astype(np.float32)
    denc_lm = np.ascontiguousarray(denc.reshape(n, 16, 2).transpose(1, 0, 2))
    gt = torch.zeros(lay.n_entries * 2, dtype=torch.float32, device="cuda")
    if variant.startswith("bucketed"):
        nb = int(L.lib().lnr_hashgrid_bwd_workspace_bytes(ctypes.byref(d), n))
        ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
    if variant == "bucketed_fwd_counts":
        table = torch.zeros(lay.n_entries * 2, dtype=torch.int16, device="cuda")
        enc = torch.empty(16, n, dtype=torch.int32, device="cuda")
        L.call("lnr_hashgrid_fwd", ctypes.byref(d), cu(pos), n, table, enc, n, ws, nb, L.stream())
        L.call("lnr_hashgrid_bwd", ctypes.byref(d), cu(pos), n, cu(denc_lm), n, gt, None, None, ws, nb, L.BWD_COUNTS_READY,
               L.stream())
    elif variant == "bucketed":
        L.call("lnr_hashgrid_bwd", ctypes.byref(d), cu(pos), n, cu(denc_lm), n, gt, None, None, ws, nb, 0, L.stream())
    else:
        L.call("lnr_hashgrid_bwd_atomic", ctypes.byref(d), cu(pos), n, cu(denc_lm), n, gt, L.stream())
    got = host(gt).reshape(-1, 2)
    ref = ohg.encode_backward(pos, denc, lay)
    err = np.linalg.norm(got - ref) / np.linalg.norm(ref)
    # fp16 record values for the binned backward (conftest.TABLE_GRAD_RTOL); fp32 atomics for the other
    assert err < (TABLE_GRAD_RTOL if variant.startswith("bucketed") else 1e-5), err
    assert np.abs(got - ref).max() < 4e-3 * np.abs(ref).max()
    # untouched entries stay exactly zero
    assert np.all(got[ref == 0] == 0)


# ------------------------------------------------------------------ sigma MLP
def _mlp_setup(rng, n):
    shapes = omlp.layer_shapes(32, 1, 64, 1)
    w0 = rng.uniform(-0.4, 0.4, shapes[0]).astype(np.float16)
    w1 = rng.uniform(-0.4, 0.4, shapes[1]).astype(np.float16)
    x = rng.uniform(-1, 1, (n, 32)).astype(np.float16)
    wflat = np.concatenate([w0.reshape(-1), w1.reshape(-1)])
    x_lm = np.ascontiguousarray(x.reshape(n, 16, 2).transpose(1, 0, 2)).view(np.int32).reshape(16, n)
    return w0, w1, x, wflat, x_lm


def test_sigma_mlp_fwd(L):
    rng = np.random.default_rng(3)
    n = 1000  # not a multiple of 16: tail tile
    w0, w1, x, wflat, x_lm = _mlp_setup(rng, n)
    sig = torch.empty(n, dtype=torch.int16, device="cuda")
    L.call("lnr_sigma_mlp_fwd", (cu(wflat.view(np.int16))), (cu(x_lm)), n, n, (sig), L.stream())
    got = host(sig).view(np.float16).astype(np.float32)
    out, _ = omlp.forward(x, [w0, w1])
    ref = out[:, 0].astype(np.float32)
    assert np.all(np.abs(got - ref) <= np.abs(ref) * 2.0 ** -9 + 2.0 ** -14), np.abs(got - ref).max()


def test_sigma_mlp_bwd(L):
    rng = np.random.default_rng(4)
    n = 4000
    w0, w1, x, wflat, x_lm = _mlp_setup(rng, n)
    dsig = (rng.normal(0, 1, n) * 10.0 ** rng.uniform(-6, 0, n)).astype(np.float32)
    # samples whose hidden pre-activation sits at 0 within fp32-vs-fp64 rounding have an ambiguous
    # ReLU mask; give them no gradient so both sides agree on every contribution
    pre = np.abs(x.astype(np.float64) @ w0.astype(np.float64).T).min(1)
    tie = pre < 1e-6
    dsig[tie] = 0.0
    denc = torch.empty(16, n, 2, dtype=torch.float32, device="cuda")
    dw = torch.zeros(3072, dtype=torch.float32, device="cuda")
    ws = torch.empty(L.lib().lnr_dw_workspace_words(n), dtype=torch.float32, device="cuda")
    L.call("lnr_sigma_mlp_bwd", (cu(wflat.view(np.int16))), (cu(x_lm)), n, n, (cu(dsig)), (denc),
           (dw), (ws), L.stream())
    out, hid = omlp.forward(x, [w0, w1])
    dout = np.zeros((n, 16))
    dout[:, 0] = dsig
    dx, dws = omlp.backward(x, [w0, w1], hid, dout)
    got_dx = host(denc).transpose(1, 0, 2).reshape(n, 32)
    # unit-d_sigma MFMA (exact fp16 operands) then fp32 scaling: fp32-accumulation accurate
    assert tie.sum() <= 3
    ok = ~tie
    per = np.where(ok, np.abs(got_dx - dx).max(1), 0)
    worst = np.argsort(per)[-6:]
    err = per.max() / np.abs(dx).max()
    assert err < 1e-5, (err, worst, per[worst], dsig[worst], pre[worst], got_dx[worst[-1]], dx[worst[-1]])
    gw = host(dw)
    ref_w = np.concatenate([dws[0].reshape(-1), dws[1].reshape(-1)])
    err = np.linalg.norm(gw - ref_w) / np.linalg.norm(ref_w)
    assert err < 2e-3, err
    assert np.all(gw[2048 + 64:] == 0)  # padded output rows get no gradient


# ------------------------------------------------------------------ sampling
def test_ogm_sampler_golden(L):
    g = np.load("tests/golden/samplers.npz")
    rays, occ = g["rays"], g["occ"]
    R = rays.shape[0]
    z = torch.empty(R, 512, dtype=torch.float32, device="cuda")
    L.call("lnr_sample_ogm", (cu(rays)), R, 512, (cu(occ)), 100, 1.0, (cu(g["u_jitter"])),
           (cu(g["u_pdf"])), 0, 0, (z), None, L.stream())
    got = host(z)
    assert np.all(np.diff(got, axis=1) >= 0)
    np.testing.assert_allclose(got, g["z_ogm"], rtol=1e-5, atol=5e-6)


def test_uniform_sampler_golden(L):
    g = np.load("tests/golden/samplers.npz")
    rays = g["rays"]
    R = rays.shape[0]
    z = torch.empty(R, 64, dtype=torch.float32, device="cuda")
    L.call("lnr_sample_uniform", (cu(rays)), R, 64, 1.0, (cu(g["u_jitter_uniform"])), 0, 0, (z),
           None, L.stream())
    np.testing.assert_allclose(host(z), g["z_uniform"], rtol=1e-6, atol=1e-7)


def test_ogm_sampler_inkernel_rng_matches_oracle(L):
    g = np.load("tests/golden/samplers.npz")
    rays, occ = g["rays"], g["occ"]
    R = rays.shape[0]
    key, off = orng.step_key(7, 3), 1000
    z = torch.empty(R, 512, dtype=torch.float32, device="cuda")
    L.call("lnr_sample_ogm", (cu(rays)), R, 512, (cu(occ)), 100, 1.0, None, None, key, off, (z),
           None, L.stream())
    a, b = orng.ray_sample_grid(np.arange(off, off + R), 256)
    uj = orng.uniform(key, orng.STREAM_JITTER, a, b)
    up = orng.uniform(key, orng.STREAM_PDF, a, b)
    ref = orender.ogm_samples(rays, 512, occ, uj, up)
    np.testing.assert_allclose(host(z), ref, rtol=1e-5, atol=5e-6)


@pytest.mark.parametrize("S", [128, 512, 2048])
@pytest.mark.parametrize("perturb", [1.0, 0.0])
def test_ogm_sampler_merge_equals_full_sort(L, S, perturb, monkeypatch):
    """The one-wave sampler's sort of the importance draws alone + one bitonic merge with the (checked
    ascending) strata (LONER_SAMPLER_MERGE=1), and the draws sorted before the inverse CDF and merged by rank
    (LONER_SAMPLER_MERGE=2, k_sampler_rank, from 256 samples), give the full bitonic sort's depths bit for bit, for
    training (jittered strata) and eval (perturb 0) draws, 2 to 32 values per lane; rays whose strata
    rounding would cross fall back to the full sort; rays with far <= near too."""
    g = np.load("tests/golden/samplers.npz")
    rays, occ = g["rays"], g["occ"]
    rng = np.random.default_rng(3)
    rays = np.concatenate([rays] * 4)
    R = rays.shape[0]
    rays[:, 11] = rng.uniform(0.0, 0.05, R)  # a spread of near / far bounds
    rays[:4, 12] = rays[:4, 11]  # far == near and far < near: no linspace estimate (the rank merge's lifting search)
    rays[4:8, 12] = rays[4:8, 11] - 0.01
    monkeypatch.setenv("LONER_SAMPLER_RANK_MIN_RAYS", "0")  # (the rank path at this test's ray count too)
    outs = []
    for m in ("0", "1", "2"):
        monkeypatch.setenv("LONER_SAMPLER_MERGE", m)
        z = torch.empty(R, S, dtype=torch.float32, device="cuda")
        L.call("lnr_sample_ogm", cu(rays), R, S, cu(occ), 100, perturb, None, None, orng.step_key(5, 2), 0, z, None,
               L.stream())
        outs.append(host(z).copy())
    np.testing.assert_array_equal(outs[0], outs[1])
    np.testing.assert_array_equal(outs[0], outs[2])
    assert np.all(np.diff(outs[2], axis=1) >= 0)


# ------------------------------------------------------------------ compositing + loss
def test_composite_default_and_adjusted_golden(L):
    g = np.load("tests/golden/composite.npz")
    rays, z, sig, noise = g["rays"], g["z"], g["sigma"], g["noise"]
    R, S = z.shape
    outs = {k: torch.empty(R, dtype=torch.float32, device="cuda") for k in ("depth", "opacity", "variance")}
    w = torch.empty(R, S, dtype=torch.float32, device="cuda")
    L.call("lnr_composite", (cu(rays)), (cu(z)), (cu(sig)), R, S, 0, 1.0, (cu(noise)), 0, 0,
           (w), (outs["depth"]), (outs["opacity"]), (outs["variance"]), L.stream())
    np.testing.assert_allclose(host(w), g["weights"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(host(outs["depth"]), g["depth"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(host(outs["opacity"]), g["opacity"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(host(outs["variance"]), g["variance"], rtol=1e-3, atol=1e-8)
    L.call("lnr_composite", (cu(rays)), (cu(z)), (cu(sig)), R, S, 1, 0.0, None, 0, 0, (w),
           (outs["depth"]), (outs["opacity"]), (outs["variance"]), L.stream())
    np.testing.assert_allclose(host(w), g["adj_weights"], rtol=1e-4, atol=1e-6)
    np.testing.assert_array_equal(host(outs["depth"]), g["adj_depth"])
    with pytest.raises(RuntimeError, match="Unknown render strategy"):
        L.call("lnr_composite", (cu(rays)), (cu(z)), (cu(sig)), R, S, 7, 0.0, None, 0, 0, None,
               (outs["depth"]), None, None, L.stream())


def _lp(L, cfg, scale, gstep, it_idx, far_ref, n_op, R, S):
    lp = L.LossParams()
    lp.kind = L.LOSS_KINDS[cfg["loss_selection"]]
    lp.scale = float(scale)
    lp.los_lambda = oloss.los_lambda(cfg, gstep)
    lp.depthloss_lambda = cfg["depthloss_lambda"]
    lp.min_depth_eps = cfg["min_depth_eps"]
    lp.min_js = cfg["JS_loss"]["min_js_score"]
    lp.max_js = cfg["JS_loss"]["max_js_score"]
    lp.js_alpha = cfg["JS_loss"]["alpha"]
    lp.los_eps = oloss.los_depth_eps(cfg, it_idx)
    lp.far_ref = float(far_ref)
    lp.inv_n_opaque = 1.0 / max(n_op, 1)
    lp.inv_rs = 1.0 / (R * S)
    lp.dev_n_opaque = None
    return lp


@pytest.mark.parametrize("tag", ["l1js_default", "l1js_haveri", "l1los", "l2js"])
def test_composite_loss_bwd_golden(L, tag):
    g = np.load(f"tests/golden/loss_{tag}.npz")
    cfg = ast.literal_eval(str(g["cfg_json"]))
    rays, z, sig, noise, dgt = g["rays"], g["z"], g["sigma"], g["noise"], g["depth_gt"]
    R, S = z.shape
    n_op = int(((dgt > 0) & ~(dgt > rays[0, -1])).sum())
    lp = _lp(L, cfg, g["scale"], int(g["global_step"]), int(g["iteration_idx"]), rays[0, -1], n_op, R, S)
    w = torch.empty(R, S, dtype=torch.float32, device="cuda")
    depth = torch.empty(R, dtype=torch.float32, device="cuda")
    op = torch.empty(R, dtype=torch.float32, device="cuda")
    dsig = torch.empty(R, S, dtype=torch.float32, device="cuda")
    stats = torch.empty(R, L.RAY_STATS, dtype=torch.float32, device="cuda")
    out = torch.empty(8, dtype=torch.float32, device="cuda")
    L.call("lnr_composite_loss_bwd", (cu(rays)), (cu(z)), (cu(sig)), (cu(dgt)), R, S, 1.0,
           (cu(noise)), 0, 0, ctypes.byref(lp), (w), (depth), (op), (dsig), (stats),
           L.stream())
    L.call("lnr_loss_finalize", (stats), R, ctypes.byref(lp), (out), L.stream())
    o = host(out)
    assert o[0] == pytest.approx(float(g["loss"]), rel=1e-4)
    assert o[1] == pytest.approx(float(g["depth_eps"]), rel=1e-5)
    np.testing.assert_allclose(host(w), g["weights"], rtol=1e-4, atol=1e-6)
    ref = g["dsigma"].reshape(R, S)
    got = host(dsig)
    err = np.abs(got - ref).max() / np.abs(ref).max()
    assert err < 1e-4, err


@pytest.mark.parametrize("replicas", [False, True])
def test_ogm_update_golden(L, replicas):
    g = np.load("tests/golden/loss_l1js_default.npz")
    occ = np.load("tests/golden/samplers.npz")["occ"]
    rays, z, dgt = g["rays"], g["z"], g["depth_gt"]
    R, S = z.shape
    grid = cu(occ.reshape(-1).copy())
    # minimum workspace: the fp32 result + one int64 copy of the grid (3 res^3 words)
    words = int(L.lib().lnr_ogm_workspace_words(100)) if replicas else 3 * grid.numel()
    ws = torch.full((words,), 7.0, device="cuda")  # garbage: the call zeroes its workspace
    L.call("lnr_ogm_update", (cu(rays)), (cu(z)), (cu(dgt)), R, S, float(g["scale"]),
           float(g["occ_lr"]), (grid), (ws), words, 100, L.stream())
    delta = host(grid) - occ.reshape(-1)
    idx = g["occ_delta_idx"]
    np.testing.assert_allclose(delta[idx], g["occ_delta"], rtol=1e-3, atol=2e-7)
    mask = np.ones(delta.size, bool)
    mask[idx] = False
    assert np.abs(delta[mask]).max() < 1e-7
    # int64 fixed-point splat: a second update from the same grid is bitwise identical
    grid2 = cu(occ.reshape(-1).copy())
    L.call("lnr_ogm_update", (cu(rays)), (cu(z)), (cu(dgt)), R, S, float(g["scale"]),
           float(g["occ_lr"]), (grid2), (ws), words, 100, L.stream())
    assert np.array_equal(host(grid2), host(grid))


# ------------------------------------------------------------------ Adam
def test_adam_matches_torch_semantics(L):
    rng = np.random.default_rng(5)
    n = 10003
    p = rng.normal(0, 1, n).astype(np.float32)
    m = np.zeros(n, np.float32)
    v = np.zeros(n, np.float32)
    tp, tm, tv = cu(np.pad(p, (0, 1))), cu(np.zeros(n + 1, np.float32)), cu(np.zeros(n + 1, np.float32))
    sh = torch.empty(n + 1, dtype=torch.float16, device="cuda")
    for step in range(1, 4):
        grad = rng.normal(0, 1e-3, n).astype(np.float32)
        ooptim.adam_step(p, grad, m, v, step, 0.01)
        L.call("lnr_adam_step", (tp), (sh), (cu(np.pad(grad, (0, 1)))), (tm), (tv), n, step,
               0.01, 0.9, 0.999, 1e-8, None, L.stream())
    np.testing.assert_allclose(host(tp)[:n], p, rtol=1e-6, atol=1e-7)
    np.testing.assert_array_equal(host(sh)[:n], host(tp)[:n].astype(np.float16))
    # torch.optim.Adam itself on the same data (CPU reference semantics)
    rng = np.random.default_rng(6)
    q = torch.nn.Parameter(torch.from_numpy(rng.normal(0, 1, 64).astype(np.float32)))
    opt = torch.optim.Adam([q], lr=0.01)
    tq = cu(q.detach().numpy().copy())
    tm2, tv2 = torch.zeros(64, device="cuda"), torch.zeros(64, device="cuda")
    for step in range(1, 6):
        gr = rng.normal(0, 1, 64).astype(np.float32)
        q.grad = torch.from_numpy(gr)
        opt.step()
        L.call("lnr_adam_step", (tq), None, (cu(gr)), (tm2), (tv2), 64, step, 0.01, 0.9, 0.999,
               1e-8, None, L.stream())
    np.testing.assert_allclose(host(tq), q.detach().numpy(), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("lvl", [3, 10])
def test_hashgrid_bwd_record_dynamic_range(L, lvl):
    """fp16 record values over a wide dynamic range (hashgrid.hpp "Record values").
    One level's encoding gradient spans 2^-30 .. 1 (log-uniform, random signs) on unsorted positions (one
    or two contributions per entry: no averaging).  The records hold w g 2^k in fp16 with 2^k = 2^9 / 2^E
    (level max < 2^E), so a contribution above 2^-23 of the level maximum is a normal fp16 (relative
    rounding 2^-11), below it a subnormal (absolute step 2^-24 scaled units) and below 2^-34 of it zero.
    Per entry, against the fp64 oracle (oracle/hashgrid.encode_backward):
      err <= 2^-11 sum|w g| + 2^-16 sum wyz |g| (tx as unorm16) + count 2^-25 2^-k (subnormal steps);
    entries whose every contribution lies below the flush threshold are exactly 0, and entries above
    2^-23 of the maximum meet the relative bar alone."""
    rng = np.random.default_rng(40 + lvl)
    n = 24000
    pos = rng.uniform(0.0, 1.0, (n, 3)).astype(np.float32)
    lay = ohg.GridLayout(16, 2, 18, 16)
    d = L.grid_desc(16, 2, 18, 16)
    denc = rng.normal(0, 1, (n, 32)).astype(np.float32)
    mag = np.exp2(rng.uniform(-30.0, 0.0, (n, 2))) * rng.choice([-1.0, 1.0], (n, 2))
    denc[:, 2 * lvl:2 * lvl + 2] = mag.astype(np.float32)
    denc_lm = np.ascontiguousarray(denc.reshape(n, 16, 2).transpose(1, 0, 2))
    nb = int(L.lib().lnr_hashgrid_bwd_workspace_bytes(ctypes.byref(d), n))
    ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
    gt = torch.zeros(lay.n_entries * 2, dtype=torch.float32, device="cuda")
    L.call("lnr_hashgrid_bwd", ctypes.byref(d), cu(pos), n, cu(denc_lm), n, gt, None, None, ws, nb, 0, L.stream())
    got = host(gt).reshape(-1, 2)
    g = denc[:, 2 * lvl:2 * lvl + 2].astype(np.float64)
    E = int(np.frexp(np.float32(np.abs(g).max()))[1])
    k = 9 - E
    w, idx = ohg.corner_weights_indices(pos, lay, lvl)
    _, frac = ohg._corners(pos, lay, lvl)
    size, off = lay.sizes[lvl], lay.offsets[lvl]
    ref = np.zeros((size, 2))
    ref_abs = np.zeros((size, 2))
    yz_abs = np.zeros((size, 2))
    cnt = np.zeros(size)
    for c in range(8):
        e = idx[:, c] - off
        wyz = (frac[:, 1] if c & 2 else 1 - frac[:, 1]) * (frac[:, 2] if c & 4 else 1 - frac[:, 2])
        np.add.at(ref, e, w[:, c:c + 1].astype(np.float64) * g)
        np.add.at(ref_abs, e, w[:, c:c + 1].astype(np.float64) * np.abs(g))
        np.add.at(yz_abs, e, wyz[:, None].astype(np.float64) * np.abs(g))
        np.add.at(cnt, e, 1.0)
    got_l = got[off:off + size].astype(np.float64)
    bound = 1.01 * 2.0 ** -11 * ref_abs + 2.0 ** -16 * yz_abs + cnt[:, None] * 2.0 ** (-25 - k) + 1e-300
    err = np.abs(got_l - ref)
    assert np.all(err <= bound), (float((err / bound).max()), int((err > bound).sum()))
    top = np.abs(g).max()
    # every record value below the flush threshold (scaled value < 2^-25 rounds to fp16 zero): exactly 0.
    # A fine level's pair record holds wyz g (the x weight applies in the accumulation): yz_abs bounds it
    below = (ref_abs > 0) & (yz_abs * 2.0 ** k < 2.0 ** -25)
    assert np.all(got_l[below] == 0.0)
    # entries above 2^-23 of the level maximum: relative (fp16 rounding + tx quantisation) bar alone
    big = ref_abs > 2.0 ** -23 * top
    assert np.all(err[big] <= 1.01 * 2.0 ** -11 * ref_abs[big] + 2.0 ** -16 * yz_abs[big] + cnt[:, None].repeat(2, 1)[big]
                  * 2.0 ** (-25 - k))
    assert big.sum() > 1000 and ((ref_abs > 0) & ~big).sum() > 100 and below.sum() > 10  # every regime occurs
    # other levels are untouched by the wide range: the usual relative L2 bar
    gall = ohg.encode_backward(pos, denc, lay)
    mask = np.ones(lay.n_entries, bool)
    mask[off:off + size] = False
    assert np.linalg.norm(got[mask] - gall[mask]) / np.linalg.norm(gall[mask]) < TABLE_GRAD_RTOL
