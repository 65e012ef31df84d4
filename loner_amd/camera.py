"""Colour-head training: the camera phase of the north-star driver.

Reference: ``Optimizer.iterate_optimizer_camera`` / ``_do_iterate_optimizer_camera`` /
``compute_loss_camera`` (src/mapping/optimizer.py:517-688,861-894), driven by
examples/fdt_optimize_implicit_map.py:826-873 (ITERATE_CAMERA) after the sigma field is trained:

* the sigma head and the poses are frozen, colour is detached from sigma
  (``detach_rgb_from_sigma``): the compositing weights are constants of the colour loss;
* a fresh ``torch.optim.Adam`` over the colour parameters (hash grid + MLP) at ``lrate_rgb`` with an
  ``ExponentialLR(lrate_gamma)`` stepped every iteration, per window;
* rays: per keyframe, a permutation of the (masked) pixels is drawn once per window and iteration
  ``it`` takes the slice [max(n*it - 1, 0), min(n*(it + 1) - 1, n_iter*n)) of it (the reference's
  own off-by-one: the first iteration has n - 1 rays per keyframe);
* loss = ``l1_loss(rgb_fine, intensities)``, a mean over 3 x rays.

One iteration here is: ``lnr_build_camera_rays`` (on the device, from the per-pixel direction table
and the resident image), the OGM sampler, the sigma encode + ``lnr_field_render`` (weights), the
colour encode (which also counts the backward's records), ``lnr_rgb_train`` (colour forward, L1
gradient, MLP backward on MFMA, d_enc), the colour hash-grid backward and Adam.  No host sync.
"""
import math
import os

import torch

from . import _lib as L


def pinhole_directions(width, height, K):
    """get_ray_directions without distortion (src/common/ray_utils.py:62-124): (H*W, 3) fp32 camera
    frame directions ((x - cx) / fx, (y - cy) / fy, 1), pixel p = y * W + x.  With distortion the
    reference undistorts the pixel grid first (calibration.undistort_points); pass that table to
    ``CameraFrames`` instead -- it is computed once per calibration, not per step."""
    xs = torch.linspace(0, width - 1, width, dtype=torch.float32)
    ys = torch.linspace(0, height - 1, height, dtype=torch.float32)
    gx, gy = torch.meshgrid(xs, ys, indexing="ij")
    gx = gx.permute(1, 0).reshape(-1, 1)
    gy = gy.permute(1, 0).reshape(-1, 1)
    K = torch.as_tensor(K, dtype=torch.float32)
    return torch.cat([(gx - K[0, 2]) / K[0, 0], (gy - K[1, 2]) / K[1, 1], torch.ones_like(gx)], -1)


class ColorState:
    """Trainable colour branch of DecoupledNeRF (nerf_tcnn.py:40-52,80-95): fp32 master parameters
    [MLP (tcnn flat) | hash table], Adam moments and the fp16 shadow the kernels read, on one GPU.
    ``head()`` returns the ``evaluate.ColorHead`` view used for rendering."""

    def __init__(self, n_hidden_layers=4, n_levels=16, log2_hashmap_size=19, base_resolution=16, device="cuda",
                 seed=1337, table_init=1e-4):
        self.device = torch.device(device)
        self.n_hidden_layers = int(n_hidden_layers)
        self.n_levels = n_levels
        self.desc = L.grid_desc(n_levels, 2, log2_hashmap_size, base_resolution, 2.0)
        self.n_entries = int(self.desc.n_entries)
        self.n_mlp = int(L.lib().lnr_rgb_mlp_params(self.n_hidden_layers))
        self.n_params = self.n_mlp + 2 * self.n_entries
        self.n_padded = (self.n_params + 3) // 4 * 4
        dev = self.device
        self.params = torch.zeros(self.n_padded, dtype=torch.float32, device=dev)
        self.grad = torch.zeros_like(self.params)
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.shadow = torch.zeros(self.n_padded, dtype=torch.float16, device=dev)
        self.adam_step = 0
        self.init_params(seed, table_init)

    def init_params(self, seed=1337, table_init=1e-4):
        """tcnn init: xavier-uniform per matrix, table U(-table_init, table_init) (counter-based draws)."""
        s = L.stream(self.device)
        shapes = [(64, 48)] + [(64, 64)] * (self.n_hidden_layers - 1) + [(16, 64)]
        off = 0
        for k, (o, i) in enumerate(shapes):
            a = math.sqrt(6.0 / (o + i))
            L.call("lnr_fill_uniform", L.ctypes.c_void_p(self.params.data_ptr() + 4 * off), o * i, seed + 1 + k,
                   -a, a, 0, s)
            off += o * i
        L.call("lnr_fill_uniform", L.ctypes.c_void_p(self.params.data_ptr() + 4 * self.n_mlp), 2 * self.n_entries,
               seed, -table_init, table_init, 0, s)
        self.refresh_shadow()

    def load(self, table, mlp):
        """Set from the reference modules' flat ``params`` (``_pos_encoding`` / ``_model_intensity``)."""
        self.params[:self.n_mlp].copy_(mlp.reshape(-1).to(self.params))
        self.params[self.n_mlp:self.n_params].copy_(table.reshape(-1).to(self.params))
        self.refresh_shadow()

    def refresh_shadow(self):
        L.call("lnr_f32_to_f16", self.params, self.shadow, self.n_padded, L.stream(self.device))

    def reset_optimizer(self):
        self.m.zero_()
        self.v.zero_()
        self.adam_step = 0

    @property
    def mlp_f16(self):
        return self.shadow[:self.n_mlp]

    @property
    def table_f16(self):
        return self.shadow[self.n_mlp:self.n_params]

    @property
    def grad_mlp(self):
        return self.grad[:self.n_mlp]

    @property
    def grad_table(self):
        return self.grad[self.n_mlp:self.n_params]

    def head(self):
        from .evaluate import ColorHead
        h = ColorHead.__new__(ColorHead)
        h.desc, h.n_hidden_layers, h.n_levels = self.desc, self.n_hidden_layers, self.n_levels
        h.table, h.mlp = self.table_f16, self.mlp_f16
        return h


class CameraFrames:
    """The keyframe window of the camera phase, resident on the device: per-pixel directions, images,
    poses and the per-window pixel permutations (optimizer.py:581-601)."""

    def __init__(self, directions, width, height, images, poses, world_cube, ray_range, masks=None,
                 n_rays_per_kf=512, seed=0, device="cuda"):
        dev = torch.device(device)
        self.device = dev
        self.width, self.height = int(width), int(height)
        self.dirs = torch.as_tensor(directions, dtype=torch.float32).reshape(-1, 3).to(dev).contiguous()
        if self.dirs.shape[0] != self.width * self.height:
            raise ValueError("directions must hold one row per pixel")
        self.images = [torch.as_tensor(im, dtype=torch.float32).reshape(self.width * self.height, -1).to(dev)
                       .contiguous() for im in images]
        self.channels = self.images[0].shape[1]
        self.poses = [torch.as_tensor(p, dtype=torch.float64).reshape(-1, 4)[:3] for p in poses]
        get = (lambda k: world_cube[k]) if isinstance(world_cube, dict) else (lambda k: getattr(world_cube, k))
        self.scale = float(torch.as_tensor(get("scale_factor")).reshape(-1)[0])
        self.shift = [float(x) for x in torch.as_tensor(get("shift")).reshape(-1)]
        self.r_min = float(ray_range[0])
        self.n = int(n_rays_per_kf)
        # FULL_CONFIG schedule (optimizer.py:581-601): n_iter = floor(min masked pixels / n); each
        # keyframe's masked pixels in a random order, the first n_iter * n of them kept
        g = torch.Generator(device="cpu").manual_seed(seed)
        pix = []
        for k in range(len(self.images)):
            idx = torch.arange(self.width * self.height)
            if masks is not None and masks[k] is not None:
                idx = idx[torch.as_tensor(masks[k]).reshape(-1).bool()]
            pix.append(idx)
        # (without masks the reference's FULL_CONFIG path cannot run -- it indexes by mask.image -- so
        # every pixel counts as unmasked here)
        self.n_iter = int(min(len(p) for p in pix) // self.n)
        keep = min(self.n_iter * self.n, min(len(p) for p in pix))
        self.perm = [p[torch.randperm(len(p), generator=g)][:keep].to(dev) for p in pix]
        self.keep = keep
        self.descs = []
        for k in range(len(self.images)):
            cam = L.CameraDesc()
            cam.width, cam.height, cam.channels = self.width, self.height, self.channels
            cam.scale, cam.r_min = self.scale, self.r_min
            for i in range(3):
                cam.shift[i] = self.shift[i]
            for i, v in enumerate(self.poses[k].reshape(-1).tolist()):
                cam.pose[i] = v
            self.descs.append(cam)
        # the window on the device for lnr_build_camera_rays_window: {camera, image} per frame, and
        # the per-frame pixel schedules as one (K, keep) array
        arr = (L.CameraFrame * len(self.images))()
        for k, img in enumerate(self.images):
            arr[k].cam = self.descs[k]
            arr[k].image = img.data_ptr()
        self.frames_dev = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
        self.perm2d = torch.stack(self.perm).contiguous() if keep > 0 else torch.zeros(len(self.images), 1,
                                                                                       dtype=torch.int64, device=dev)

    def iteration_slice(self, it):
        """[max(n*it - 1, 0), min(n*(it + 1) - 1, n_iter*n)) (optimizer.py:633-635)."""
        lo = max(self.n * it - 1, 0)
        hi = min(self.n * (it + 1) - 1, self.keep)
        return lo, hi

    def n_rays(self, it):
        lo, hi = self.iteration_slice(it)
        return len(self.images) * max(hi - lo, 0)

    def build(self, it, rays, intensities):
        """Camera rays + intensities of iteration ``it`` for every keyframe, concatenated in keyframe
        order (optimizer.py:614-655).  Returns the ray count."""
        lo, hi = self.iteration_slice(it)
        n = max(hi - lo, 0)
        L.call("lnr_build_camera_rays_window", self.frames_dev, len(self.images), self.dirs, self.perm2d, self.keep, lo,
               n, rays, intensities, L.stream(self.device))  # every keyframe in one launch
        return len(self.images) * n


class CameraStepEngine:
    """One colour-head optimiser iteration on preallocated workspaces for up to ``n_rays`` rays."""

    def __init__(self, field, color: ColorState, n_rays, n_samples=512, perturb=1.0, raw_noise_std=1.0,
                 lr=0.01, gamma=1.0, seed=0, allreduce=None, ray_offset=0, skip_zero=None):
        if n_samples % 64:
            raise ValueError(f"n_samples={n_samples} must be a multiple of 64")
        self.field, self.color = field, color
        self.R, self.S = int(n_rays), int(n_samples)
        self.perturb, self.noise_std = float(perturb), float(raw_noise_std)
        self.lr, self.gamma, self.seed = float(lr), float(gamma), int(seed)
        self.allreduce, self.ray_offset = allreduce, int(ray_offset)
        # (None: LONER_CAM_SKIP_ZERO, default on)
        self.skip_zero = (os.environ.get("LONER_CAM_SKIP_ZERO", "1") == "1") if skip_zero is None else bool(skip_zero)
        # with skip_zero: the live encode also counts the backward's records (by the weights' mask), so the
        # backward needs no counting pass of its own (LONER_CAM_LIVE_COUNT, default on)
        self.live_count = self.skip_zero and os.environ.get("LONER_CAM_LIVE_COUNT", "1") == "1"
        self.iteration = 0
        dev = field.device
        N = self.R * self.S
        self.N = N
        self.z = torch.empty(self.R, self.S, dtype=torch.float32, device=dev)
        self.enc = torch.empty(field.cfg.n_levels, N, dtype=torch.int32, device=dev)
        self.enc_rgb = torch.empty(color.n_levels, N, dtype=torch.int32, device=dev)
        self.d_enc = torch.empty(color.n_levels, N, 2, dtype=torch.float32, device=dev)
        self.weights = torch.empty(self.R, self.S, dtype=torch.float32, device=dev)
        self.depth = torch.empty(self.R, dtype=torch.float32, device=dev)
        self.opacity = torch.empty(self.R, dtype=torch.float32, device=dev)
        self.rgb = torch.empty(self.R, 3, dtype=torch.float32, device=dev)
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self.bwd_ws_bytes = int(L.lib().lnr_hashgrid_bwd_workspace_bytes(L.ctypes.byref(color.desc), N))
        self.bwd_ws = torch.empty(self.bwd_ws_bytes, dtype=torch.uint8, device=dev)
        # the colour backward's per-level max |d_enc| (record scales), written by lnr_rgb_train
        self.level_max_ptr = L.ctypes.c_void_p(L.lib().lnr_hashgrid_bwd_level_max(L.ctypes.byref(color.desc), N,
                                                                                   L.ptr(self.bwd_ws)))
        self.ws_bytes = int(L.lib().lnr_rgb_train_workspace_bytes(color.n_hidden_layers, self.R))
        self.ws = torch.empty(self.ws_bytes, dtype=torch.uint8, device=dev)

    def colour_encode(self, rays, R, S, s):
        """The colour grid's encode of the R x S samples (after the sigma pass wrote ``weights``).
        skip_zero: samples of weight exactly 0 have no colour gradient (dL/dc_i = w_i dL/drgb): no gathers
        for them (nor zero stores in tiles without a live sample), and no records in the backward at the
        levels that are not coherent.  Round 4 measured it slower at CAM (encode 0.34 -> 0.21 ms, backward
        0.90 -> 0.99 ms); with round 5's kernels the encode drops 0.285 -> 0.19 ms and the backward stays
        0.452-0.458 -> 0.456-0.463: CAM 1.806 -> 1.708 ms.  On by default.  live_count: the live encode
        counts the backward's records too (the backward's own counting pass was 0.12 ms at CAM)."""
        cs = self.color
        if self.live_count:
            L.call("lnr_hashgrid_fwd_rays_live_ws", L.ctypes.byref(cs.desc), rays, self.z, R, S, cs.table_f16,
                   self.weights, self.enc_rgb, self.N, self.bwd_ws, self.bwd_ws_bytes, s)
        elif self.skip_zero:
            L.call("lnr_hashgrid_fwd_rays_live", L.ctypes.byref(cs.desc), rays, self.z, R, S, cs.table_f16,
                   self.weights, self.enc_rgb, self.N, s)
        else:
            L.call("lnr_hashgrid_fwd_rays", L.ctypes.byref(cs.desc), rays, self.z, R, S, cs.table_f16, self.enc_rgb,
                   self.N, self.bwd_ws, self.bwd_ws_bytes, s)

    def colour_grid_backward(self, rays, R, S, s):
        """The colour table's gradient from ``d_enc`` (lnr_rgb_train's output), in colour_encode's mode."""
        cs = self.color
        if self.skip_zero:  # records of live samples only: counted by the encode (live_count) or here
            flags = (L.BWD_COUNTS_READY if self.live_count else 0) | L.BWD_LEVEL_MAX_READY
            L.call("lnr_hashgrid_bwd_rays_live", L.ctypes.byref(cs.desc), rays, self.z, R, S, self.d_enc, self.N,
                   self.weights, cs.grad_table, self.bwd_ws, self.bwd_ws_bytes, flags, s)
        else:
            L.call("lnr_hashgrid_bwd_rays", L.ctypes.byref(cs.desc), rays, self.z, R, S, self.d_enc, self.N,
                   cs.grad_table, None, None, self.bwd_ws, self.bwd_ws_bytes,
                   L.BWD_COUNTS_READY | L.BWD_LEVEL_MAX_READY, s)

    def step(self, rays, intensities, global_step=None, n_rays_global=None):
        """rays (R,13), intensities (R,3) on the GPU, R <= n_rays.  Returns the loss (device, local
        rays' share when data-parallel)."""
        fs, cs = self.field, self.color
        R, S = rays.shape[0], self.S
        if R > self.R:
            raise ValueError(f"{R} rays exceed the engine capacity {self.R}")
        if intensities.shape[-1] != 3:
            raise ValueError("the colour loss needs 3 intensity channels (num_colors = 3)")
        N = self.N
        s = L.stream(fs.device)
        gstep = self.iteration if global_step is None else int(global_step)
        key = int(L.lib().lnr_step_key(self.seed, gstep))
        if fs.cfg.sampler == "OGM":
            L.call("lnr_sample_ogm", rays, R, S, fs.occ, fs.cfg.occ_res, self.perturb, None, None, key,
                   self.ray_offset, self.z, None, s)
        else:
            L.call("lnr_sample_uniform", rays, R, S, self.perturb, None, key, self.ray_offset, self.z, None, s)
        L.call("lnr_hashgrid_fwd_rays", L.ctypes.byref(fs.desc), rays, self.z, R, S, fs.table_f16, self.enc, N,
               None, 0, s)
        L.call("lnr_field_render", fs.mlp_f16, self.enc, N, rays, self.z, R, S, 0, self.noise_std, None, key,
               self.ray_offset, self.depth, self.opacity, None, self.weights, s)
        self.colour_encode(rays, R, S, s)
        n_glob = R if n_rays_global is None else int(n_rays_global)
        L.call("lnr_rgb_train", cs.mlp_f16, cs.n_hidden_layers, self.enc_rgb, N, rays, self.weights, intensities, R,
               S, 1.0 / (3.0 * n_glob), self.rgb, self.loss, self.d_enc, cs.grad_mlp, self.ws, self.ws_bytes,
               self.level_max_ptr, s)
        self.colour_grid_backward(rays, R, S, s)
        if self.allreduce is not None:
            self.allreduce(cs.grad)
        cs.adam_step += 1
        lr = self.lr * self.gamma ** (cs.adam_step - 1)  # ExponentialLR stepped once per iteration
        L.call("lnr_adam_step", cs.params, cs.shadow, cs.grad, cs.m, cs.v, cs.n_padded, cs.adam_step, lr, 0.9,
               0.999, 1e-8, None, s)
        self.iteration += 1
        return self.loss
