"""Dump lnr_field_train's MLP-backward outputs (dW0, dW1, J = dsigma/denc, d_enc, level maxima) for one
seeded synthetic batch, so two libraries can be compared bit for bit (GPU box):
    LONER_AMD_LIB=a.so python tools/mlp_bwd_dump.py out_a.npz
    LONER_AMD_LIB=b.so python tools/mlp_bwd_dump.py out_b.npz
    python tools/mlp_bwd_dump.py --compare out_a.npz out_b.npz
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    for k in A.files:
        x, y = A[k], B[k]
        same = np.array_equal(x.view(np.uint32) if x.dtype == np.float32 else x,
                              y.view(np.uint32) if y.dtype == np.float32 else y)
        n_diff = int((x != y).sum())
        rel = float(np.linalg.norm((x - y).astype(np.float64)) / max(np.linalg.norm(x.astype(np.float64)), 1e-30))
        print(f"{k:6s} bitwise={same} differing={n_diff}/{x.size} rel_l2={rel:.3e}")


def main():
    if sys.argv[1] == "--compare":
        return compare(sys.argv[2], sys.argv[3])
    import torch
    from loner_amd import _lib as L
    dev = torch.device("cuda", 0)
    R, S = 256, 512
    rng = np.random.default_rng(5)
    w0 = rng.uniform(-0.5, 0.5, (64, 32)).astype(np.float16)
    w1 = (rng.uniform(-0.2, 1.0, (16, 64)) * 8).astype(np.float16)
    x = rng.uniform(-1, 1, (R * S, 32)).astype(np.float16)
    rays = np.zeros((R, 13), np.float32)
    d = rng.normal(0, 1, (R, 3))
    rays[:, 3:6] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 12] = 10.0
    z = np.sort(rng.uniform(0.5, 10.0, (R, S)), 1).astype(np.float32)
    dgt = rng.uniform(1.0, 9.0, R).astype(np.float32)
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    wflat = np.concatenate([w0.reshape(-1), w1.reshape(-1)]).view(np.int16)
    x_lm = np.ascontiguousarray(x.reshape(-1, 16, 2).transpose(1, 0, 2)).view(np.int32).reshape(16, -1)
    lp = L.LossParams()
    lp.kind = L.LOSS_KINDS["L2_JS"]
    lp.scale, lp.los_lambda, lp.depthloss_lambda = 0.1, 100.0, 0.005
    lp.min_depth_eps, lp.min_js, lp.max_js, lp.js_alpha, lp.los_eps = 0.5, 0.1, 10.0, 1.0, 3.0
    lp.far_ref, lp.inv_n_opaque, lp.inv_rs, lp.dev_n_opaque = 10.0, 1.0 / R, 1.0 / (R * S), None
    f32 = lambda *s: torch.zeros(*s, dtype=torch.float32, device=dev)
    d_enc, d_w = f32(16, R * S, 2), f32(3072)
    ws = f32(L.lib().lnr_field_train_workspace_words(R, S))
    stats, depth, op, w, lmax = f32(R, L.RAY_STATS), f32(R), f32(R), f32(R, S), f32(16)
    jac = torch.zeros(16, R * S, dtype=torch.int32, device=dev)
    out = {}
    for name, dj in (("enc", None), ("jac", jac)):
        d_w.zero_()
        L.call("lnr_field_train", cu(wflat), cu(x_lm), R * S, cu(rays), cu(z), cu(dgt), R, S, 0.0, None, 0, 0,
               ctypes.byref(lp), d_enc, d_w, ws, stats, depth, op, w, lmax, dj, L.stream())
        torch.cuda.synchronize()
        gw = d_w.cpu().numpy().copy()
        out[f"dW0_{name}"], out[f"dW1_{name}"] = gw[:2048], gw[2048:]
        out[f"lmax_{name}"] = lmax.cpu().numpy().copy()
    out["d_enc"] = d_enc.cpu().numpy()
    out["jac"] = jac.cpu().numpy()
    np.savez(sys.argv[1], **out)
    print("wrote", sys.argv[1], {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
