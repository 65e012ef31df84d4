"""ctypes binding of the C ABI in ``include/loner_amd.h`` (``loner_amd/_lib/libloner_amd.so``).

The library is built in-tree by ``python -m loner_amd.build`` (or ``__graft_entry__.build()``).
There is no fallback: if the library is missing or a call fails, a RuntimeError is raised —
mirroring tiny-cuda-nn's ``CHECK_THROW`` behaviour at the same boundary.

torch is imported before the library is loaded so that the library binds to the HIP runtime
torch already loaded (one runtime per process; streams are shared).
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the dlopen, see module docstring)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libloner_amd.so")
# Kernel experiments load an alternative in-tree build (tools/exp_variants.py); unset in production.
LIB_PATH = os.environ.get("LONER_AMD_LIB", LIB_PATH)
MAX_LEVELS = 32
RAY_STATS = 5
SIGMA_MLP_PARAMS = 64 * 32 + 16 * 64

LOSS_KINDS = {"L1_JS": 0, "L2_JS": 1, "L1_LOS": 2, "L2_LOS": 3}
RENDER_STRATEGIES = {"default": 0, "adjusted": 1}
BWD_COUNTS_READY = 1
BWD_NO_ACCUM = 2
BWD_LEVEL_MAX_READY = 4
BWD_LIVE = 8  # the live backward: records only for samples with d_sigma != 0 (bitwise the full one)
BWD_PREPARE_ONLY = 16  # stop before the scatter (histogram + scans); needs BWD_LIVE or BWD_COUNTS_READY
BWD_PREPARED = 32  # a BWD_PREPARE_ONLY call with the same arguments ran

c_p = ctypes.c_void_p
c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_u32 = ctypes.c_uint32
c_f = ctypes.c_float
c_d = ctypes.c_double


class GridDesc(ctypes.Structure):
    _fields_ = [("n_levels", ctypes.c_uint32), ("n_features", ctypes.c_uint32),
                ("log2_hashmap_size", ctypes.c_uint32), ("base_resolution", ctypes.c_uint32),
                ("per_level_scale", ctypes.c_float), ("n_entries", ctypes.c_uint32),
                ("scale", ctypes.c_float * MAX_LEVELS), ("resolution", ctypes.c_uint32 * MAX_LEVELS),
                ("size", ctypes.c_uint32 * MAX_LEVELS), ("offset", ctypes.c_uint32 * (MAX_LEVELS + 1))]


class StepScalars(ctypes.Structure):
    """``lnr_step_scalars``: the per-step scalars a captured step reads from device memory."""
    _fields_ = [("key", ctypes.c_uint32), ("los_lambda", ctypes.c_float), ("los_eps", ctypes.c_float),
                ("adam_step_size", ctypes.c_float), ("adam_bc2_sqrt", ctypes.c_float), ("pad", ctypes.c_uint32 * 3)]


class AdamRange(ctypes.Structure):
    """lnr_adam_range (include/loner_amd.h)."""
    _fields_ = [("param", ctypes.c_void_p), ("shadow", ctypes.c_void_p), ("grad", ctypes.c_void_p),
                ("m", ctypes.c_void_p), ("v", ctypes.c_void_p), ("n", ctypes.c_int64)]


ADAM_MAX_RANGES = 8


class AdamEpilogue(ctypes.Structure):
    """lnr_adam_epilogue (include/loner_amd.h): Adam fused into the hash-grid backward."""
    _fields_ = [("param", ctypes.c_void_p), ("shadow", ctypes.c_void_p), ("m", ctypes.c_void_p), ("v", ctypes.c_void_p),
                ("step", ctypes.c_int32), ("lr", ctypes.c_double), ("beta1", ctypes.c_double),
                ("beta2", ctypes.c_double), ("eps", ctypes.c_double), ("dev_step", ctypes.c_void_p)]


class LossParams(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("scale", ctypes.c_float), ("los_lambda", ctypes.c_float),
                ("depthloss_lambda", ctypes.c_float), ("min_depth_eps", ctypes.c_float),
                ("min_js", ctypes.c_float), ("max_js", ctypes.c_float), ("js_alpha", ctypes.c_float),
                ("los_eps", ctypes.c_float), ("far_ref", ctypes.c_float), ("inv_n_opaque", ctypes.c_float),
                ("inv_rs", ctypes.c_float), ("dev_n_opaque", ctypes.c_void_p), ("dev_far_ref", ctypes.c_void_p),
                ("dev_status", ctypes.c_void_p), ("dev_loss_out", ctypes.c_void_p), ("flags", ctypes.c_int32),
                ("dev_step", ctypes.c_void_p), ("dev_d_ray", ctypes.c_void_p), ("dev_term_hist", ctypes.c_void_p)]


LP_DW_OVERWRITE = 1
LP_SIGMA_READY = 2
LP_FORWARD_ONLY = 4
LP_BACKWARD_ONLY = 8


STATUS_NAN_LOSS, STATUS_INF_LOSS, STATUS_SIGMA_CLIPPED, STATUS_NONFINITE_OUTPUT = 1, 2, 4, 8


SELECT = {"RANDOM": 0, "MASK": 1, "ALL": 2, "GIVEN": 3}


class RayWindowDesc(ctypes.Structure):
    """``lnr_ray_window``: device pointers of a resident keyframe window (loner_amd.rays.RayWindow)."""
    _fields_ = [("n_kf", ctypes.c_int32), ("scale", ctypes.c_float), ("shift", ctypes.c_float * 3),
                ("r_min", ctypes.c_float), ("r_max", ctypes.c_float), ("poses", c_p), ("dirs", c_p), ("dists", c_p),
                ("scan_off", c_p), ("order", c_p), ("n_trunk", c_p), ("sky_dirs", c_p), ("sky_off", c_p),
                ("ray_off", c_p), ("n_sel", c_p), ("n_sel_trunk", c_p), ("dev_step", c_p)]


class MotionComp(ctypes.Structure):
    """``lnr_motion_comp``."""
    _fields_ = [("start_rot", ctypes.c_float * 9), ("start_t", ctypes.c_float * 3), ("delta_t", ctypes.c_float * 3),
                ("axis", ctypes.c_float * 3), ("angle", ctypes.c_float), ("t0", ctypes.c_float), ("t1", ctypes.c_float),
                ("target_inv", ctypes.c_float * 12), ("identity", ctypes.c_int32)]


class CameraDesc(ctypes.Structure):
    """``lnr_camera_desc``."""
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("channels", ctypes.c_int32),
                ("scale", ctypes.c_float), ("shift", ctypes.c_float * 3), ("r_min", ctypes.c_float),
                ("pose", ctypes.c_float * 12)]


class CameraFrame(ctypes.Structure):
    """``lnr_camera_frame``."""
    _fields_ = [("cam", CameraDesc), ("image", ctypes.c_void_p)]


class SkyParams(ctypes.Structure):
    """``lnr_sky_params``."""
    _fields_ = [("rot", ctypes.c_float * 9), ("top_rows", ctypes.c_int32), ("horizon_deg", ctypes.c_float)]


_SIGNATURES = {
    "lnr_version": (ctypes.c_int, []),
    "lnr_last_error": (ctypes.c_char_p, []),
    "lnr_grid_desc_init": (ctypes.c_int, [ctypes.POINTER(GridDesc), c_u32, c_u32, c_u32, c_u32, c_f]),
    "lnr_hashgrid_fwd": (ctypes.c_int, [ctypes.POINTER(GridDesc), c_p, c_i64, c_p, c_p, c_i64, c_p, c_i64, c_p]),
    "lnr_hashgrid_fwd_rays": (ctypes.c_int, [ctypes.POINTER(GridDesc), c_p, c_p, c_i64, c_i32, c_p, c_p, c_i64, c_p,
                                             c_i64, c_p]),
    "lnr_hashgrid_bwd_workspace_bytes": (c_i64, [ctypes.POINTER(GridDesc), c_i64]),
    "lnr_hashgrid_bwd_level_max": (c_p, [ctypes.POINTER(GridDesc), c_i64, c_p]),
    "lnr_hashgrid_bwd_seg_start": (c_p, [ctypes.POINTER(GridDesc), c_i64, c_p]),
    "lnr_hashgrid_bwd": (ctypes.c_int, [ctypes.POINTER(GridDesc), c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p, c_i64,
                                        c_i32, c_p]),
    "lnr_hashgrid_bwd_rays": (ctypes.c_int, [ctypes.POINTER(GridDesc), c_p, c_p, c_i64, c_i32, c_p, c_i64, c_p, c_p,
                                             c_p, c_p, c_i64, c_i32, c_p]),
    "lnr_hashgrid_bwd_rays_jac": (ctypes.c_int, [ctypes.POINTER(GridDesc), c_p, c_p, c_i64, c_i32, c_p, c_p, c_i64,
                                                 c_p, c_p, c_p, c_p, c_i64, c_i32, c_p]),
    "lnr_hashgrid_bwd_rays_jac_adam": (ctypes.c_int, [ctypes.POINTER(GridDesc), c_p, c_p, c_i64, c_i32, c_p, c_p, c_i64,
                                                      ctypes.POINTER(AdamEpilogue), c_p, c_i64, c_i32, c_p]),
    "lnr_hashgrid_bwd_accum": (ctypes.c_int, [ctypes.POINTER(GridDesc), c_i64, c_p, c_i64, c_u32, c_u32, c_p, c_p]),
    "lnr_hashgrid_bwd_accum_flags": (ctypes.c_int, [ctypes.POINTER(GridDesc), c_i64, c_p, c_i64, c_u32, c_u32, c_p,
                                                     ctypes.c_int32, c_p]),
    "lnr_hashgrid_bwd_atomic": (ctypes.c_int, [ctypes.POINTER(GridDesc), c_p, c_i64, c_p, c_i64, c_p, c_p]),
    "lnr_hashgrid_bwd_rays_atomic": (ctypes.c_int, [ctypes.POINTER(GridDesc), c_p, c_p, c_i64, c_i32, c_p, c_i64, c_p,
                                                    c_p]),
    "lnr_enc_to_aos": (ctypes.c_int, [c_p, c_i64, c_i64, c_u32, c_p, c_p]),
    "lnr_aos_grad_to_enc": (ctypes.c_int, [c_p, c_p, c_i64, c_u32, c_p, c_i64, c_p]),
    "lnr_sh_encode": (ctypes.c_int, [c_p, c_i64, c_i32, c_p, c_p]),
    "lnr_sigma_mlp_fwd": (ctypes.c_int, [c_p, c_p, c_i64, c_i64, c_p, c_p]),
    "lnr_dw_workspace_words": (c_i64, [c_i64]),
    "lnr_field_train_workspace_words": (c_i64, [c_i64, c_i32]),
    "lnr_sigma_mlp_bwd": (ctypes.c_int, [c_p, c_p, c_i64, c_i64, c_p, c_p, c_p, c_p, c_p]),
    "lnr_step_key": (c_u32, [c_u32, c_u32]),
    "lnr_sample_ogm": (ctypes.c_int, [c_p, c_i64, c_i32, c_p, c_i32, c_f, c_p, c_p, c_u32, c_i64, c_p, c_p, c_p]),
    "lnr_sample_uniform": (ctypes.c_int, [c_p, c_i64, c_i32, c_f, c_p, c_u32, c_i64, c_p, c_p, c_p]),
    "lnr_composite": (ctypes.c_int, [c_p, c_p, c_p, c_i64, c_i32, c_i32, c_f, c_p, c_u32, c_i64, c_p, c_p, c_p, c_p,
                                     c_p]),
    "lnr_composite_bwd": (ctypes.c_int, [c_p, c_p, c_p, c_i64, c_i32, c_i32, c_f, c_p, c_u32, c_i64, c_p, c_p, c_p,
                                         c_p, c_p, c_p, c_p]),
    "lnr_composite_loss_bwd": (ctypes.c_int, [c_p, c_p, c_p, c_p, c_i64, c_i32, c_f, c_p, c_u32, c_i64,
                                              ctypes.POINTER(LossParams), c_p, c_p, c_p, c_p, c_p, c_p]),
    "lnr_field_train": (ctypes.c_int, [c_p, c_p, c_i64, c_p, c_p, c_p, c_i64, c_i32, c_f, c_p, c_u32, c_i64,
                                       ctypes.POINTER(LossParams), c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p,
                                       c_p]),
    "lnr_field_sigma_phase": (ctypes.c_int, [c_p, c_p, c_i64, c_p, c_p, c_i64, c_i32, c_i32, c_i32, c_f, c_p, c_u32,
                                             c_i64, ctypes.POINTER(LossParams), c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "lnr_pose_grad": (ctypes.c_int, [c_p, c_p, c_p, c_p, c_i64, c_i32, c_p, c_i64, c_p, c_p, c_p, c_i32, c_f, c_f, c_p,
                                     c_p, c_p]),
    "lnr_pose_adam": (ctypes.c_int, [c_p, c_p, c_p, c_p, c_p, c_i32, c_i64, c_f, c_f, c_f, c_f, c_p, c_p]),
    "lnr_field_render": (ctypes.c_int, [c_p, c_p, c_i64, c_p, c_p, c_i64, c_i32, c_i32, c_f, c_p, c_u32, c_i64, c_p,
                                        c_p, c_p, c_p, c_p]),
    "lnr_rgb_render": (ctypes.c_int, [c_p, c_i32, c_p, c_i64, c_p, c_p, c_i64, c_i32, c_p, c_p]),
    "lnr_hashgrid_fwd_rays_phase": (ctypes.c_int, [ctypes.POINTER(GridDesc), c_p, c_p, c_i64, c_i32, c_p, c_p, c_i64,
                                                   c_p, c_i64, c_p, c_p, c_i64, c_i32, c_i32, c_p]),
    "lnr_hashgrid_fwd_rays_live": (ctypes.c_int, [ctypes.POINTER(GridDesc), c_p, c_p, c_i64, c_i32, c_p, c_p, c_p, c_i64,
                                                  c_p]),
    "lnr_hashgrid_fwd_rays_live_ws": (ctypes.c_int, [ctypes.POINTER(GridDesc), c_p, c_p, c_i64, c_i32, c_p, c_p, c_p,
                                                     c_i64, c_p, c_i64, c_p]),
    "lnr_hashgrid_bwd_rays_live": (ctypes.c_int, [ctypes.POINTER(GridDesc), c_p, c_p, c_i64, c_i32, c_p, c_i64, c_p, c_p,
                                                  c_p, c_i64, c_i32, c_p]),
    "lnr_status_scan": (ctypes.c_int, [c_p, c_i64, c_u32, c_p, c_p]),
    "lnr_rgb_mlp_params": (c_i64, [c_i32]),
    "lnr_rgb_train_workspace_bytes": (c_i64, [c_i32, c_i64]),
    "lnr_rgb_train": (ctypes.c_int, [c_p, c_i32, c_p, c_i64, c_p, c_p, c_p, c_i64, c_i32, c_f, c_p, c_p, c_p, c_p,
                                     c_p, c_i64, c_p, c_p]),
    "lnr_build_camera_rays": (ctypes.c_int, [ctypes.POINTER(CameraDesc), c_p, c_p, c_p, c_i64, c_p, c_p, c_p]),
    "lnr_build_camera_rays_window": (ctypes.c_int, [c_p, c_i32, c_p, c_p, c_i64, c_i64, c_i64, c_p, c_p, c_p]),
    "lnr_motion_compensate": (ctypes.c_int, [ctypes.POINTER(MotionComp), c_p, c_p, c_p, c_i64, c_p]),
    "lnr_sky_rays_capacity": (c_i64, []),
    "lnr_sky_rays": (ctypes.c_int, [c_p, c_i64, ctypes.POINTER(SkyParams), c_p, c_i64, c_p, c_p]),
    "lnr_loss_finalize": (ctypes.c_int, [c_p, c_i64, ctypes.POINTER(LossParams), c_p, c_p]),
    "lnr_count_opaque": (ctypes.c_int, [c_p, c_i64, c_f, c_p, c_p, c_p]),
    "lnr_build_lidar_rays": (ctypes.c_int, [ctypes.POINTER(RayWindowDesc), c_i32, c_p, c_u32, c_i64, c_i64, c_p, c_p,
                                            c_p, c_p, c_p, c_p]),
    "lnr_adam_step": (ctypes.c_int, [c_p, c_p, c_p, c_p, c_p, c_i64, c_i32, c_d, c_d, c_d, c_d, c_p, c_p]),
    "lnr_adam_step_ranges": (ctypes.c_int, [c_p, c_i32, c_i32, c_d, c_d, c_d, c_d, c_p, c_p]),
    "lnr_step_scalars_set": (ctypes.c_int, [c_p, c_i32, c_p, c_p]),
    "lnr_adam_coefficients": (ctypes.c_int, [c_i32, c_d, c_d, c_d, ctypes.POINTER(c_f), ctypes.POINTER(c_f)]),
    "lnr_ogm_workspace_words": (c_i64, [c_i32]),
    "lnr_ogm_update": (ctypes.c_int, [c_p, c_p, c_p, c_i64, c_i32, c_f, c_f, c_p, c_p, c_i64, c_i32, c_p]),
    "lnr_ogm_grad": (ctypes.c_int, [c_p, c_p, c_p, c_i64, c_i32, c_f, c_p, c_i64, c_i32, c_p]),
    "lnr_grid_sample3d": (ctypes.c_int, [c_p, c_i32, c_p, c_i64, c_p, c_p]),
    "lnr_grid_sample3d_bwd_workspace_words": (c_i64, [c_i32]),
    "lnr_grid_sample3d_bwd": (ctypes.c_int, [c_p, c_p, c_i64, c_i32, c_p, c_p, c_i64, c_p]),
    "lnr_sgd_step": (ctypes.c_int, [c_p, c_p, c_i64, c_f, c_p]),
    "lnr_fill_uniform": (ctypes.c_int, [c_p, c_i64, c_u32, c_f, c_f, c_i64, c_p]),
    "lnr_f32_to_f16": (ctypes.c_int, [c_p, c_p, c_i64, c_p]),
}

_lib = None


def lib():
    """Load (once) and return the ctypes library; raises RuntimeError if it is not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"loner_amd: HIP library not built ({LIB_PATH}); run `python -m loner_amd.build`")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, what=""):
    if rc != 0:
        msg = lib().lnr_last_error().decode(errors="replace")
        raise RuntimeError(f"{what}: {msg}" if what else msg)


def call(name, *args):
    """Call a C-ABI entry point; torch tensors are passed as device pointers.  The tensors stay
    referenced for the duration of the call; afterwards the caching allocator's stream ordering
    keeps their memory valid for the enqueued kernels."""
    conv = [ptr(a) if isinstance(a, torch.Tensor) else a for a in args]
    rc = getattr(lib(), name)(*conv)
    check(rc, name)
    return rc


def ptr(t):
    """Device pointer of a tensor (or None -> NULL).  The tensor must be contiguous and on the GPU."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("loner_amd: expected a GPU tensor (the HIP path has no CPU fallback)")
    if not t.is_contiguous():
        raise RuntimeError("loner_amd: expected a contiguous tensor")
    return ctypes.c_void_p(t.data_ptr())


def stream(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def grid_desc(n_levels=16, n_features=2, log2_hashmap_size=18, base_resolution=16, per_level_scale=2.0):
    d = GridDesc()
    check(lib().lnr_grid_desc_init(ctypes.byref(d), n_levels, n_features, log2_hashmap_size, base_resolution,
                                   per_level_scale), "lnr_grid_desc_init")
    return d


def step_key(seed, step):
    return int(lib().lnr_step_key(seed & 0xFFFFFFFF, step & 0xFFFFFFFF))


def exported_symbols():
    return sorted(_SIGNATURES)
