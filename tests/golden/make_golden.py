"""Generate golden vectors by running the REFERENCE's own pure-torch code (build container only).

Usage (needs /root/reference, which never travels to the GPU box):
    python tests/golden/make_golden.py          # writes tests/golden/*.npz

The reference imports tinycudann / open3d / pytorch3d / kornia / torchviz / attrdict at module
level; none is needed by the functions exercised here, so they are replaced by inert stub
modules.  All random draws (stratified jitter, inverse-CDF u, sigma noise)
are generated here with numpy, fed to the reference through a patched ``torch.rand`` /
``torch.randn`` and stored next to the outputs so that the oracle and the HIP path can be fed
the identical draws.  Fixtures are data only (inputs + expected outputs).
"""
import importlib.abc
import importlib.machinery
import os
import sys
import types
from types import SimpleNamespace as NS

import numpy as np
import torch

REF = os.environ.get("LONER_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
STUBS = ("tinycudann", "torchviz", "open3d", "pytorch3d", "kornia", "attrdict", "cv2", "rosbag",
         "rospy", "cv_bridge", "sensor_msgs", "ros_numpy", "tf2_msgs", "geometry_msgs", "std_msgs", "tf2_py",
         "nav_msgs")
# modules the reference imports that do not exist in its own tree (analysis.fdt_common_utils)
STUB_PREFIXES = ("analysis.fdt_common_utils",)


class _Anything(types.ModuleType):
    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        sub = _Anything(f"{self.__name__}.{name}")
        setattr(self, name, sub)
        return sub

    def __call__(self, *a, **k):
        return _Anything(self.__name__ + "()")


class _StubFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def find_spec(self, name, path, target=None):
        if name.split(".")[0] in STUBS or name.startswith(STUB_PREFIXES):
            return importlib.machinery.ModuleSpec(name, self, is_package=True)
        return None

    def create_module(self, spec):
        m = _Anything(spec.name)
        m.__path__ = []
        if spec.name == "attrdict":
            m.AttrDict = type("AttrDict", (dict,), {})
        return m

    def exec_module(self, module):
        pass


def import_reference():
    sys.meta_path.insert(0, _StubFinder())
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REF, "src"))
    import models.rendering_tcnn as rendering
    import models.losses as losses
    import models.ray_sampling as ray_sampling
    import models.model_tcnn as model_tcnn
    import mapping.optimizer as optimizer
    import common.ray_utils as ray_utils
    import common.pose_utils as pose_utils
    return NS(rendering=rendering, losses=losses, ray_sampling=ray_sampling, model_tcnn=model_tcnn,
              optimizer=optimizer, ray_utils=ray_utils, pose_utils=pose_utils)


class DrawQueue:
    """Patches torch.rand / torch.randn to return pre-generated draws in call order."""

    def __init__(self, draws):
        self.draws = list(draws)
        self._rand, self._randn = torch.rand, torch.randn

    def _pop(self, *size, **kw):
        if len(size) == 1 and isinstance(size[0], (tuple, list, torch.Size)):
            size = tuple(size[0])
        d = self.draws.pop(0)
        assert tuple(d.shape) == tuple(size), (d.shape, size)
        return torch.from_numpy(d.copy()).to(kw.get("dtype") or torch.float32)

    def __enter__(self):
        torch.rand = self._pop
        torch.randn = self._pop
        return self

    def __exit__(self, *a):
        torch.rand, torch.randn = self._rand, self._randn
        assert not self.draws, f"{len(self.draws)} unused draws"


def u24(rng, shape):
    return (rng.integers(0, 1 << 24, size=shape) * 2.0 ** -24).astype(np.float32)


def synthetic_rays(ref, rng, n, cube_scale, cube_shift, ray_range, pose_t, n_sky=0, zero_depth=0):
    """Rays from the reference's own LidarRayDirections.build_lidar_rays on a random scan."""
    el = rng.uniform(-0.6, 0.6, n)
    az = rng.uniform(-np.pi, np.pi, n)
    dirs = np.stack([np.cos(el) * np.cos(az), np.cos(el) * np.sin(az), np.sin(el)]).astype(np.float32)
    dist = rng.uniform(ray_range[0] + 1.0, ray_range[1] * 0.8, n).astype(np.float32)
    if zero_depth:
        dist[:zero_depth] = 0.0
    if n_sky:
        dist[-n_sky:] = ray_range[1] + 1.0
    scan = NS(ray_directions=torch.from_numpy(dirs), distances=torch.from_numpy(dist),
              timestamps=torch.zeros(n))
    wc = ref.pose_utils.WorldCube(torch.tensor([cube_scale], dtype=torch.float32),
                                  torch.tensor(cube_shift, dtype=torch.float32))
    pose = torch.eye(4)
    pose[:3, 3] = torch.tensor(pose_t)
    rd = ref.ray_utils.LidarRayDirections(scan)
    rays, depths = rd.build_lidar_rays(torch.arange(n), torch.tensor(ray_range, dtype=torch.float32), wc, pose)
    return dirs, dist, pose.numpy(), rays.numpy(), depths.numpy()


def sigma_profiles(rng, z, depth_gt, far):
    """fp16-valued sigma (R,S): peaked, multi-modal, empty, negative, saturated."""
    R, S = z.shape
    sig = np.zeros((R, S), np.float32)
    for r in range(R):
        kind = r % 6
        d = depth_gt[r] if 0 < depth_gt[r] < far[r] else z[r, S // 2]
        width = (rng.uniform(0.002, 0.01))
        if kind in (0, 1):
            sig[r] = rng.uniform(200, 3000) * np.exp(-0.5 * ((z[r] - d) / width) ** 2)
        elif kind == 2:
            d2 = z[r, int(S * 0.3)]
            sig[r] = 800 * np.exp(-0.5 * ((z[r] - d) / width) ** 2) + 400 * np.exp(-0.5 * ((z[r] - d2) / width) ** 2)
        elif kind == 3:
            sig[r] = 0.0
        elif kind == 4:
            sig[r] = rng.normal(-2.0, 5.0, S)
        else:
            sig[r] = np.where(np.abs(z[r] - d) < width, 65504.0, rng.uniform(0, 3, S))
    return sig.astype(np.float16).astype(np.float32)


LOSS_DEFAULT = dict(loss_selection="L1_JS", JS_loss=dict(min_js_score=1.0, max_js_score=10.0, alpha=1.0),
                    decay_los_lambda=False, los_lambda=1000.0, min_los_lambda=10.0, los_lambda_decay_rate=0.001,
                    los_lambda_decay_steps=15000, decay_depth_eps=True, depth_eps=3.0, min_depth_eps=0.5,
                    depth_eps_decay_rate=0.95, depth_eps_decay_steps=1, depthloss_lambda=0.005)
LOSS_HAVERI = dict(LOSS_DEFAULT, JS_loss=dict(min_js_score=0.1, max_js_score=10.0, alpha=1.0),
                   decay_los_lambda=True, los_lambda_decay_rate=0.0001, depth_eps_decay_steps=100)


def _ns(d):
    return NS(**{k: (_ns(v) if isinstance(v, dict) else v) for k, v in d.items()})


class FixedSigmaModel(torch.nn.Module):
    """Stand-in for DecoupledNeRF: returns a stored sigma leaf (the tcnn field is not importable)."""

    def __init__(self, sigma):
        super().__init__()
        self.sigma = torch.nn.Parameter(sigma)

    def forward(self, xyz, d, sigma_only, detach_sigma):
        assert xyz.shape[0] == self.sigma.numel()
        return self.sigma.reshape(-1, 1)


class FixedZSampler:
    def __init__(self, z):
        self.z = z

    def get_samples(self, rays, n, perturb):
        return self.z


def make_optimizer(ref, loss_cfg, scale, sampler, sigma, n_samples, occ=None, occ_lr=1e-4, global_step=0):
    Opt = ref.optimizer.Optimizer
    o = Opt.__new__(Opt)
    model = ref.model_tcnn.Model.__new__(ref.model_tcnn.Model)
    torch.nn.Module.__init__(model)
    model.cfg = _ns(dict(render=dict(N_samples_train=n_samples, N_samples_test=n_samples, perturb=1.0, chunk=16384,
                                     retraw=True, raw_noise_std=1.0, netchunk=0), ray_range=[1, 75], num_colors=3))
    model.nerf_model = FixedSigmaModel(sigma)
    o._model = model
    o._ray_sampler = sampler
    o._scale_factor = torch.tensor([scale], dtype=torch.float32)
    o._device = "cpu"
    o._model_config = _ns(dict(loss=loss_cfg, model=dict(occ_model=dict(N_iters_acc=10, lr=occ_lr))))
    o._settings = _ns(dict(debug=dict(visualize_loss=False, draw_samples=False, draw_rays_eps=False, store_ray=False)))
    o._optimization_settings = ref.optimizer.OptimizationSettings()
    o._global_step = global_step
    o._keyframe_count = 0
    if occ is not None:
        om = ref.model_tcnn.OccupancyGridModel.__new__(ref.model_tcnn.OccupancyGridModel)
        torch.nn.Module.__init__(om)
        om.occupancy_grid = torch.nn.Parameter(torch.from_numpy(occ.copy()).reshape(1, 1, *occ.shape))
        o._occupancy_grid_model = om
        o._occupancy_grid = om()
        o._occupancy_grid_optimizer = torch.optim.SGD(om.parameters(), lr=occ_lr)
    return o


def smooth_occ(rng, n=100):
    g = rng.normal(0, 1, (n // 10 + 2,) * 3)
    g = torch.nn.functional.interpolate(torch.from_numpy(g)[None, None], size=(n, n, n), mode="trilinear",
                                        align_corners=False)[0, 0].numpy()
    return (np.round(3.0 * g * 16) / 16).astype(np.float32)  # 1/16 lattice: compresses well


def main():
    ref = import_reference()
    rng = np.random.default_rng(20240807)
    torch.set_num_threads(4)
    quad_scale, quad_shift = 121.426537, [-22.5, 5.0, -3.5]
    hav_scale, hav_shift = 116.75345611572266, [-10.527198791503906, 89.2310791015625, 4.763427734375]

    # ---- rays: build_lidar_rays / get_far_val (ray_utils.py:31-60, 269-322)
    dirs, dist, pose, rays, depths = synthetic_rays(ref, rng, 96, hav_scale, hav_shift, [2.5, 45.0], [1.0, -2.0, 0.5],
                                                    n_sky=8, zero_depth=4)
    far_unclipped = ref.ray_utils.get_far_val(torch.from_numpy(rays[:, :3]), torch.from_numpy(rays[:, 3:6]), True).numpy()
    np.savez_compressed(f"{OUT}/rays.npz", dirs=dirs, dist=dist, pose=pose, scale=np.float32(hav_scale),
                        shift=np.float32(hav_shift), ray_range=np.float32([2.5, 45.0]), rays=rays, depths=depths,
                        far_val=far_unclipped)

    # ---- world cubes (pose_utils.py:222-314), bbox branch
    cubes = {}
    for name, bbox, rr in [("quad", dict(x=[-5, 50], y=[-25, 15], z=[-3, 10]), [1, 75]),
                           ("haveri_bbox", dict(x=[-10, 10], y=[-10, 10], z=[-10, 10]), [2.5, 45])]:
        wc = ref.pose_utils.compute_world_cube(None, None, None, None, rr, padding=0.3, traj_bounding_box=bbox)  # callers: loner.py:104, fdt driver :232
        cubes[name] = np.concatenate([wc.scale_factor.numpy().reshape(1), wc.shift.numpy().reshape(3)]).astype(np.float32)
    np.savez_compressed(f"{OUT}/world_cube.npz", **cubes)

    # ---- sample_pdf (rendering_tcnn.py:19-68)
    R = 24
    bins = np.sort(rng.uniform(0.01, 0.6, (R, 255)).astype(np.float32), 1)
    w = rng.uniform(0, 1, (R, 254)).astype(np.float32)
    w[::4] = 0.0
    w[1::4, 100:140] = 0.0
    u = u24(rng, (R, 256))
    with DrawQueue([u]):
        samples = ref.rendering.sample_pdf(torch.from_numpy(bins), torch.from_numpy(w), 256, det=False).numpy()
    np.savez_compressed(f"{OUT}/sample_pdf.npz", bins=bins, weights=w, u=u, samples=samples)

    # ---- samplers (ray_sampling.py:18-92) + grid_sample (model_tcnn.py:126-134)
    occ = smooth_occ(rng)
    occ[:, :, :30] = -20.0
    R = 32
    rays_s = rays[:R].copy()
    uj, up = u24(rng, (R, 256)), u24(rng, (R, 256))
    samp = ref.ray_sampling.OccGridRaySampler()
    samp.update_occ_grid(torch.from_numpy(occ).reshape(1, 1, 100, 100, 100))
    with DrawQueue([uj, up]):
        z_ogm = samp.get_samples(torch.from_numpy(rays_s), 512, 1.0).numpy()
    uj2 = u24(rng, (R, 64))
    with DrawQueue([uj2]):
        z_uni = ref.ray_sampling.UniformRaySampler().get_samples(torch.from_numpy(rays_s), 64, 1.0).numpy()
    pts = rng.uniform(-1.05, 1.05, (R, 37, 3)).astype(np.float32)
    interp = ref.model_tcnn.OccupancyGridModel.interpolate(torch.from_numpy(occ).reshape(1, 1, 100, 100, 100),
                                                           torch.from_numpy(pts)).numpy()
    np.savez_compressed(f"{OUT}/samplers.npz", rays=rays_s, occ=occ, u_jitter=uj, u_pdf=up, z_ogm=z_ogm,
                        u_jitter_uniform=uj2, z_uniform=z_uni, pts=pts, interp=interp)

    # ---- raw2outputs default + adjusted (rendering_tcnn.py:70-295)
    depth_gt = depths[:R]
    far = rays_s[:, -1]
    sig = sigma_profiles(rng, z_ogm, depth_gt, far)
    noise = rng.normal(0, 1, sig.shape).astype(np.float32)
    with DrawQueue([noise]):
        rgb, d, wts, op, var = ref.rendering.raw2outputs(torch.from_numpy(sig)[..., None], torch.from_numpy(z_ogm),
                                                         torch.from_numpy(rays_s[:, 3:6]), 1.0, True, sigma_only=True,
                                                         far=torch.from_numpy(rays_s[:, -1:]), ret_var=True)
    ad = ref.rendering.raw2outputs_adjusted(torch.from_numpy(sig)[..., None], torch.from_numpy(z_ogm),
                                            torch.from_numpy(rays_s[:, :3]), torch.from_numpy(rays_s[:, 3:6]), 1.0, True,
                                            sigma_only=True, far=torch.from_numpy(rays_s[:, -1:]), ret_var=True)
    np.savez_compressed(f"{OUT}/composite.npz", rays=rays_s, z=z_ogm, sigma=sig, noise=noise, weights=wts.numpy(),
                        depth=d.numpy(), opacity=op.numpy(), variance=var.numpy(), adj_weights=ad[2].numpy(),
                        adj_depth=ad[1].numpy(), adj_opacity=ad[3].numpy(), adj_variance=ad[4].numpy())

    # ---- compute_loss (optimizer.py:701-859) + _step_occupancy_grid (:897-908)
    for tag, cfg, scale, gstep in [("l1js_default", LOSS_DEFAULT, hav_scale, 0),
                                   ("l1js_haveri", LOSS_HAVERI, hav_scale, 1234),
                                   ("l1los", dict(LOSS_DEFAULT, loss_selection="L1_LOS"), hav_scale, 7),
                                   ("l2js", dict(LOSS_DEFAULT, loss_selection="L2_JS"), hav_scale, 3)]:
        uj, up = u24(rng, (R, 256)), u24(rng, (R, 256))
        noise = rng.normal(0, 1, (R, 512)).astype(np.float32)
        samp = ref.ray_sampling.OccGridRaySampler()
        samp.update_occ_grid(torch.from_numpy(occ).reshape(1, 1, 100, 100, 100))
        with DrawQueue([uj, up]):
            z = samp.get_samples(torch.from_numpy(rays_s), 512, 1.0).numpy()
        sig = torch.from_numpy(sigma_profiles(rng, z, depth_gt, far))
        it_idx = 5
        o = make_optimizer(ref, cfg, scale, samp, sig.clone(), 512, occ=occ, occ_lr=1e-3, global_step=gstep)
        with DrawQueue([uj, up, noise]):
            loss = o.compute_loss(None, (torch.from_numpy(rays_s), torch.from_numpy(depth_gt)), it_idx)
        loss.backward()
        g32 = o._model.nerf_model.sigma.grad.numpy().copy()
        res = {k: v.detach().numpy() for k, v in o._results_lidar.items() if isinstance(v, torch.Tensor) and v.numel() > 1}
        depth_eps = o._depth_eps
        o._step_occupancy_grid()
        occ_new = o._occupancy_grid.detach().numpy().reshape(100, 100, 100)
        # fp64 gradient reference on the same z / sigma / noise
        o64 = make_optimizer(ref, cfg, scale, FixedZSampler(torch.from_numpy(z).double()), sig.clone().double(), 512,
                             global_step=gstep)
        with DrawQueue([noise.astype(np.float64)]):
            loss64 = o64.compute_loss(None, (torch.from_numpy(rays_s).double(), torch.from_numpy(depth_gt).double()), it_idx)
        loss64.backward()
        delta_idx = np.flatnonzero(occ_new != occ)
        np.savez_compressed(f"{OUT}/loss_{tag}.npz", rays=rays_s, depth_gt=depth_gt, u_jitter=uj, u_pdf=up,
                            noise=noise, sigma=sig.numpy(), z=z, weights=res["weights_fine"], depth=res["depth_fine"],
                            opacity=res["opacity_fine"], variance=res["variance"], loss=np.float64(loss.item()),
                            loss64=np.float64(loss64.item()), dsigma=g32, dsigma64=o64._model.nerf_model.sigma.grad.numpy(),
                            depth_eps=np.float64(depth_eps), occ_delta_idx=delta_idx,
                            occ_delta=(occ_new.reshape(-1)[delta_idx] - occ.reshape(-1)[delta_idx]), scale=np.float32(scale),
                            global_step=np.int64(gstep), iteration_idx=np.int64(it_idx), occ_lr=np.float32(1e-3),
                            cfg_json=np.array(repr(cfg)))

    # ---- losses.py helpers (get_weights_gt :29-51, get_logits_grad :54-62) and JS (:913-925)
    s = np.sort(rng.uniform(0, 60, (16, 128)).astype(np.float32), 1)
    g = rng.uniform(5, 50, (16, 1)).astype(np.float32)
    eps = rng.uniform(0.5, 5.5, (16, 1)).astype(np.float32)
    wgt = ref.losses.get_weights_gt(torch.from_numpy(s), torch.from_numpy(g), torch.from_numpy(eps)).numpy()
    lg = ref.losses.get_logits_grad(torch.from_numpy(s), torch.from_numpy(g)).numpy()
    Opt = ref.optimizer.Optimizer
    o = Opt.__new__(Opt)
    m2 = rng.uniform(5, 50, (16, 1)).astype(np.float32)
    s2 = rng.uniform(0.01, 10, (16, 1)).astype(np.float32)
    js = o.calculate_JS_divergence(torch.from_numpy(g), 0.5 / 3.0, torch.from_numpy(m2), torch.from_numpy(s2)).numpy()
    np.savez_compressed(f"{OUT}/loss_helpers.npz", s=s, g=g, eps=eps, weights_gt=wgt, logits_grad=lg, m2=m2, s2=s2, js=js)
    print("golden vectors written to", OUT)


# ---------------------------------------------------------------------------------------------
# Round-2 fixtures (``python tests/golden/make_golden.py r2``): the camera phase and colour
# compositing, the camera loss and its colour gradient, torch.optim.Adam on tcnn-style fp16 params,
# and the checkpoint's key layout.  They go to their own files; main()'s fixtures are not touched.

def _tcnn_shape_stub():
    """A shape-only tinycudann stand-in: each module owns a flat ``params`` Parameter on the meta
    device, sized by loner_amd.tcnn's restatement of tcnn v1.7's parameter counts (so the SIZES in
    the key fixture are this build's formulas; the KEYS and module paths are the reference's)."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    from loner_amd import tcnn as ltc
    m = types.ModuleType("tinycudann")

    class _Base(torch.nn.Module):
        dtype = torch.half

        def __init__(self, n):
            super().__init__()
            self.params = torch.nn.Parameter(torch.empty(n, device="meta"))

    class Encoding(_Base):
        def __init__(self, n_input_dims, encoding_config, seed=1337, dtype=torch.half):
            cfg = dict(encoding_config)
            n = ltc._GridSpec(n_input_dims, cfg).n_params if cfg.get("otype") == "HashGrid" else 0
            super().__init__(n)
            self.n_output_dims = n_input_dims if cfg.get("otype") != "HashGrid" else \
                int(cfg["n_levels"]) * int(cfg["n_features_per_level"])
            if cfg.get("otype") == "SphericalHarmonics":
                self.n_output_dims = int(cfg["degree"]) ** 2

    class Network(_Base):
        def __init__(self, n_input_dims, n_output_dims, network_config, seed=1337):
            super().__init__(ltc._MLPSpec(n_input_dims, n_output_dims, dict(network_config)).n_params)

    class NetworkWithInputEncoding(_Base):
        def __init__(self, n_input_dims, n_output_dims, encoding_config, network_config, seed=1337):
            g = ltc._GridSpec(n_input_dims, dict(encoding_config))
            mlp = ltc._MLPSpec(g.n_levels * g.n_features, n_output_dims, dict(network_config))
            super().__init__(mlp.n_params + g.n_params)

    m.Encoding, m.Network, m.NetworkWithInputEncoding = Encoding, Network, NetworkWithInputEncoding
    return m


class FixedColorModel(torch.nn.Module):
    """Stand-in for Model in compute_loss_camera: per-sample colours are a leaf Parameter, composited
    by the reference's own raw2outputs (white background, sigma_only=False) with fixed sigma, z and
    noise, so autograd gives the loss gradient with respect to the colours."""

    def __init__(self, ref, colors, sigma, z, far):
        super().__init__()
        self.ref, self.colors = ref, torch.nn.Parameter(colors)
        self.sigma, self.z, self.far = sigma, z, far

    def forward(self, rays, sampler, scale, camera=True, return_variance=True):
        raw = torch.cat([self.colors, self.sigma[..., None]], -1)
        rgb, depth, w, op, var = self.ref.rendering.raw2outputs(raw, self.z, rays[:, 3:6], 1.0, True, sigma_only=False,
                                                                far=self.far, ret_var=True)
        return {"rgb_fine": rgb, "depth_fine": depth, "weights_fine": w}


def main_r2():
    import yaml
    sys.modules["tinycudann"] = _tcnn_shape_stub()
    ref = import_reference()
    rng = np.random.default_rng(20261016)
    torch.set_num_threads(4)

    # ---- camera rays: get_ray_directions (ray_utils.py:62-124, no distortion) and
    #      CameraRayDirections.build_rays (:175-212)
    W, H = 40, 24
    K = torch.tensor([[31.5, 0.0, 19.25], [0.0, 30.0, 11.75], [0.0, 0.0, 1.0]])
    dirs, gx, gy = ref.ray_utils.get_ray_directions(H, W, newK=K, with_indices=True)
    crd = ref.ray_utils.CameraRayDirections.__new__(ref.ray_utils.CameraRayDirections)
    crd.directions, crd.i_meshgrid, crd.j_meshgrid = dirs, gx, gy
    a, b = 0.6, -0.3
    Rz = torch.tensor([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]], dtype=torch.float32)
    Rx = torch.tensor([[1, 0, 0], [0, np.cos(b), -np.sin(b)], [0, np.sin(b), np.cos(b)]], dtype=torch.float32)
    T = torch.eye(4)
    T[:3, :3] = Rz @ Rx
    T[:3, 3] = torch.tensor([3.0, -7.5, 1.25])
    pose = NS(get_transformation_matrix=lambda: T.clone())
    wc = ref.pose_utils.WorldCube(torch.tensor([37.5]), torch.tensor([-2.0, 4.0, 0.5]))
    img = torch.from_numpy(rng.uniform(0, 1, (H, W, 3)).astype(np.float32))
    pix = torch.from_numpy(rng.choice(W * H, 300, replace=False))
    rays_c, inten = crd.build_rays(pix, pose, NS(image=img), wc, torch.tensor([1.0, 75.0]))
    np.savez_compressed(f"{OUT}/camera_rays.npz", K=K.numpy(), width=np.int64(W), height=np.int64(H),
                        directions=dirs.numpy(), grid_x=gx.numpy(), grid_y=gy.numpy(), pose=T.numpy(),
                        scale=np.float32(37.5), shift=np.float32([-2.0, 4.0, 0.5]), ray_range=np.float32([1.0, 75.0]),
                        image=img.numpy(), pixels=pix.numpy(), rays=rays_c.numpy(), intensities=inten.numpy())

    # ---- colour compositing, white background (rendering_tcnn.py:219-295 with sigma_only=False), and
    #      compute_loss_camera (optimizer.py:861-894) with its gradient w.r.t. the per-sample colours
    R, S = 48, 64
    rays = rays_c[:R].clone()
    z = torch.sort(torch.from_numpy(rng.uniform(0.02, 0.9, (R, S)).astype(np.float32)), 1).values
    far = rays[:, -1:].clone()
    sig = torch.from_numpy(sigma_profiles(rng, z.numpy(), (z[:, S // 3]).numpy(), far[:, 0].numpy()))
    col = torch.from_numpy(rng.uniform(0.0, 1.0, (R, S, 3)).astype(np.float16).astype(np.float32))
    noise = rng.normal(0, 1, (R, S)).astype(np.float32)
    with DrawQueue([noise]):
        rgb, depth, wts, op, var = ref.rendering.raw2outputs(torch.cat([col, sig[..., None]], -1), z, rays[:, 3:6], 1.0,
                                                             True, sigma_only=False, far=far, ret_var=True)
    gt = torch.from_numpy(rng.uniform(0, 1, (R, 3)).astype(np.float32))
    o = make_optimizer(ref, LOSS_DEFAULT, 37.5, None, sig.clone(), S)
    o._model = FixedColorModel(ref, col.clone(), sig, z, far)
    with DrawQueue([noise]):
        loss = o.compute_loss_camera((rays, gt), None, 0)
    loss.backward()
    np.savez_compressed(f"{OUT}/camera_loss.npz", rays=rays.numpy(), z=z.numpy(), sigma=sig.numpy(), colors=col.numpy(),
                        noise=noise, rgb=rgb.numpy(), depth=depth.numpy(), weights=wts.numpy(), opacity=op.numpy(),
                        gt=gt.numpy(), loss=np.float64(loss.item()), d_colors=o._model.colors.grad.numpy())

    # ---- torch.optim.Adam on tcnn-style fp16 params (optimizer.py:257-265,460; Adam defaults), the
    #      gradient arriving as tcnn's binding hands it over: computed with the loss scaled by 128,
    #      stored fp16, then divided by 128 (in fp16).  The same steps on an fp32 Parameter fed the
    #      identical fp16-rounded gradients (the fp32 master this build keeps) are stored beside it.
    n, steps = 4096, 5
    p0 = rng.uniform(-1e-4, 1e-4, n).astype(np.float32)
    p0[:64] = rng.uniform(-0.3, 0.3, 64)  # MLP-like weights
    graw = np.stack([rng.normal(0, 1, n) * 10.0 ** rng.uniform(-8, -2, n) for _ in range(steps)]).astype(np.float32)
    graw[:, 3000:] = 0.0  # untouched table entries
    g16 = ((torch.from_numpy(graw) * 128.0).half() / 128.0)  # fp16, as tcnn's binding returns it
    out = {}
    for tag, dt in (("fp16", torch.float16), ("fp32", torch.float32)):
        prm = torch.nn.Parameter(torch.from_numpy(p0.copy()).to(dt))  # (a copy: .to(float32) would alias p0)
        opt = torch.optim.Adam([prm], lr=0.01)
        hist = []
        for k in range(steps):
            prm.grad = g16[k].to(dt)
            opt.step()
            hist.append(prm.detach().float().numpy().copy())
        out[f"params_{tag}"] = np.stack(hist)
        out[f"exp_avg_sq_{tag}"] = opt.state[prm]["exp_avg_sq"].float().numpy()
    np.savez_compressed(f"{OUT}/adam_fp16.npz", p0=p0, grad_raw=graw, grad_f16=g16.float().numpy(), lr=np.float32(0.01),
                        **out)

    # ---- checkpoint key layout: the reference's Model / OccupancyGridModel state_dict keys
    nerf_cfg = yaml.safe_load(open(os.path.join(REF, "cfg", "nerf_config", "default_nerf_hash.yaml")))
    model = ref.model_tcnn.Model(NS(model_type="nerf_decoupled", nerf_config=nerf_cfg, num_colors=3))
    occ = ref.model_tcnn.OccupancyGridModel(NS(voxel_size=100))
    import json
    keys = dict(network_state_dict={k: list(v.shape) for k, v in model.state_dict().items()},
                occ_model_state_dict={k: list(v.shape) for k, v in occ.state_dict().items()},
                sigma_parameters=[n for n, _ in model.nerf_model._model_sigma.named_parameters()],
                note="keys and module paths from the reference's Model; sizes from the shape-only tcnn stand-in "
                     "(loner_amd.tcnn's restatement of tcnn v1.7's parameter counts)")
    json.dump(keys, open(f"{OUT}/ckpt_keys.json", "w"), indent=1, sort_keys=True)
    print("round-2 golden vectors written to", OUT)

# ---------------------------------------------------------------------------------------------
# Round-3 fixtures (``python tests/golden/make_golden.py r3``): the C5 submap pipeline.  The
# reference's own examples/fdt_segment_and_optimize_submaps.py is imported (ROS / open3d stubbed)
# and run on the committed haveri keyframe trajectory: its split + padding loop writes one trajectory
# CSV per submap and calls optimize_implicit_map, which is replaced by a recorder.  Each written CSV
# then goes through the driver's own world-cube branch for submaps
# (examples/fdt_optimize_implicit_map.py:208-233): build_poses_from_df(df, False) and
# compute_world_cube(camera_to_lidar=None, ..., padding=0.3, submap=name) (the hpk dataset family has no
# calibration object: examples/utils.py:119-123).  A second, synthetic trajectory whose middle part is
# shorter than the 30-pose padding records that the reference raises there.

class _SettingsStub(dict):
    """Settings.load_from_file / augment stand-in for the segmentation loop, which only reads
    experiment_name and system.log_dir_prefix (fdt_segment_and_optimize_submaps.py:52-67)."""
    log_dir = None

    @classmethod
    def load_from_file(cls, path):
        return cls()

    def augment(self, changes):
        pass

    def __getattr__(self, k):
        if k == "system":
            return NS(log_dir_prefix=_SettingsStub.log_dir)
        return self[k]


def _run_reference_segmentation(seg, tum, workdir, tag):
    import shutil
    import yaml
    d = os.path.join(workdir, tag)
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(d)
    traj = os.path.join(d, "gt.txt")
    with open(traj, "w") as f:
        for row in tum:
            f.write(" ".join(repr(float(v)) for v in row) + "\n")
    cfg = os.path.join(d, "run.yaml")
    yaml.safe_dump(dict(baseline="defaults.yaml", changes=None, experiment_name=tag, groundtruth_traj=traj), open(cfg, "w"))
    _SettingsStub.log_dir = d
    calls = []
    seg.Settings = _SettingsStub
    seg.optimize_implicit_map = lambda exp_dir, cfg_path, submap=None: calls.append(submap)
    err = None
    try:
        seg.optimize_and_segment_implicit_map(cfg)
    except IndexError as e:  # a neighbouring part shorter than the padding
        err = repr(e)
    files = sorted(os.listdir(os.path.join(d, tag, "trajectories"))) if os.path.isdir(os.path.join(d, tag, "trajectories")) else []
    return d, tag, calls, files, err


def main_r3():
    import pandas as pd
    ref = import_reference()
    sys.path.insert(0, os.path.join(REF, "analysis"))
    import examples.fdt_segment_and_optimize_submaps as seg
    work = os.path.join(os.path.dirname(os.path.dirname(OUT)), "scratch", "golden_r3")
    tum = np.load(f"{OUT}/haveri_keyframe_trajectory.npz")["tum"]
    d, tag, calls, files, err = _run_reference_segmentation(seg, tum, work, "haveri")
    assert err is None, err
    tdir = os.path.join(d, tag, "trajectories")
    names, rows, scales, shifts, mid = [], [], [], [], []
    ts_index = {float(t): i for i, t in enumerate(tum[:, 0])}
    for fn in files:
        df = pd.read_csv(os.path.join(tdir, fn), names=["timestamp", "x", "y", "z", "q_x", "q_y", "q_z", "q_w"],
                         delimiter=" ")
        idx = np.array([ts_index[float(t)] for t in df["timestamp"]])
        poses, _ = ref.pose_utils.build_poses_from_df(df, False)
        wc = ref.pose_utils.compute_world_cube(None, None, None, poses, (2.5, 45.0), padding=0.3, submap=fn[:-4])
        names.append(fn[:-4])
        rows.append(idx)
        scales.append(float(wc.scale_factor.reshape(-1)[0]))
        shifts.append(wc.shift.numpy().reshape(3))
    mids = np.load(os.path.join(d, tag, "submaps_middlepoints.npy"))
    offsets = np.cumsum([0] + [len(r) for r in rows])
    # a trajectory whose second part is shorter than the padding: 0.9 m steps, then 2.6 m steps
    steps = np.concatenate([np.full(55, 0.9), np.full(25, 2.6), np.full(70, 0.9)])
    xyz = np.stack([np.concatenate([[0.0], np.cumsum(steps)]), np.zeros(len(steps) + 1), np.zeros(len(steps) + 1)], 1)
    short = np.concatenate([np.arange(len(xyz))[:, None] * 0.1, xyz, np.tile([0.0, 0.0, 0.0, 1.0], (len(xyz), 1))], 1)
    _, _, calls_s, files_s, err_s = _run_reference_segmentation(seg, short, work, "short")
    np.savez_compressed(f"{OUT}/submaps.npz", names=np.array(names), row_index=np.concatenate(rows),
                        row_offsets=offsets, scale=np.float32(scales), shift=np.float32(shifts), middle_points=mids,
                        ray_range=np.float32([2.5, 45.0]), short_tum=short, short_raises=np.bool_(err_s is not None),
                        short_files_written=np.int64(len(files_s)), short_calls=np.int64(len(calls_s)))
    print("round-3 golden vectors written to", OUT, names, scales, err_s, files_s, calls_s)


# ---------------------------------------------------------------------------------------------
# Round-4 fixtures (``python tests/golden/make_golden.py r4``): every branch of compute_world_cube
# (src/common/pose_utils.py:131-149,222-314), in particular the camera-frustum branch the fdt driver
# takes with a Fusion Portable calibration (examples/fdt_optimize_implicit_map.py:195-233).  The
# Fusion Portable calibration files are dataset files (not in the reference), so the camera is a
# synthetic one of the same shape: K of a 1024 x 768 camera at im_scale_factor 0.5, a lidar-to-camera
# extrinsic rotating the lidar's x axis onto the camera's -z axis, plus a small offset.  Poses: the
# committed haveri keyframe trajectory through build_poses_from_df (zero_origin True for whole runs,
# False for submaps, as the driver does at :208-213).

def main_r4():
    import pandas as pd
    ref = import_reference()
    tum = np.load(f"{OUT}/haveri_keyframe_trajectory.npz")["tum"][:240]
    df = pd.DataFrame(tum, columns=["timestamp", "x", "y", "z", "q_x", "q_y", "q_z", "q_w"])
    poses_zero, _ = ref.pose_utils.build_poses_from_df(df, True)
    poses_raw, _ = ref.pose_utils.build_poses_from_df(df, False)
    K = torch.tensor([[303.3, 0.0, 258.0], [0.0, 303.1, 193.25], [0.0, 0.0, 1.0]])
    image_size = (384, 512)  # (height, width), as the driver passes it
    R = torch.tensor([[0.0, -1.0, 0.0], [0.0, 0.0, 1.0], [-1.0, 0.0, 0.0]])  # lidar x -> camera -z
    l2c = torch.eye(4)
    l2c[:3, :3] = R
    l2c[:3, 3] = torch.tensor([0.05, -0.12, 0.08])
    c2l = l2c.inverse()
    n = poses_raw.shape[0]
    Ks = K.expand(n, 3, 3).clone()
    Ks[:, 0, 0] += torch.linspace(0, 5, n)
    sizes = torch.tensor(image_size, dtype=torch.float32).expand(n, 2).clone()
    sizes[n // 2:] = torch.tensor([360.0, 480.0])
    bbox = dict(x=[-5.0, 50.0], y=[-25.0, 15.0], z=[-3.0, 10.0])
    cases = {
        "camera_rebased": (c2l, K, image_size, poses_zero, (1.0, 50.0), 0.3, None, None),
        "camera_submap_per_pose": (c2l, Ks, sizes, poses_raw, (1.0, 50.0), 0.3, None, "submap_1"),
        "lidar_rebased": (None, None, None, poses_zero, (2.5, 45.0), 0.3, None, None),
        "bbox_camera": (c2l, K, image_size, None, (1.0, 50.0), 0.3, bbox, None),
        "bbox_lidar": (None, None, None, None, (1.0, 75.0), 0.3, bbox, None),
    }
    out = dict(tum=tum, K=K.numpy(), Ks=Ks.numpy(), image_size=np.float32(image_size), sizes=sizes.numpy(),
               camera_to_lidar=c2l.numpy(), bbox=np.float32([bbox["x"], bbox["y"], bbox["z"]]))
    for name, (c, k, hw, poses, rr, pad, bb, sub) in cases.items():
        wc = ref.pose_utils.compute_world_cube(c, k, hw, poses, rr, padding=pad, traj_bounding_box=bb, submap=sub)
        out[f"{name}_scale"] = np.float32(wc.scale_factor.reshape(-1)[0])
        out[f"{name}_shift"] = wc.shift.numpy().reshape(3).astype(np.float32)
        print(name, float(wc.scale_factor.reshape(-1)[0]), wc.shift.numpy())
    np.savez_compressed(f"{OUT}/world_cube_camera.npz", **out)
    print("round-4 golden vectors written to", OUT)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "r2":
        main_r2()
    elif len(sys.argv) > 1 and sys.argv[1] == "r3":
        main_r3()
    elif len(sys.argv) > 1 and sys.argv[1] == "r4":
        main_r4()
    else:
        main()
