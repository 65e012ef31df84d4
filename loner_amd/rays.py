"""World cube and LiDAR ray construction (host-side data preparation feeding the hot path).

Mirrors the reference's interface and semantics:
  WorldCube                ``src/common/pose_utils.py:23-57``
  compute_world_cube       ``src/common/pose_utils.py:131-149,222-314`` (every branch: camera
                           frustums or LiDAR cube, ground-truth poses or trajectory bbox, submaps)
  get_far_val              ``src/common/ray_utils.py:31-60``
  LidarRayDirections       ``src/common/ray_utils.py:252-322`` (13-column rays, 1 m validity filter)
  build_keyframe_rays      ``KeyFrame.build_lidar_rays`` ``src/mapping/keyframe.py:75-105`` (+ sky rays)
The reference runs this on the CPU (``data_prep_on_cpu: True``, cfg/defaults.yaml:39); these
torch implementations run on whatever device their inputs live on.  On-device ray selection and
building is SURVEY §8(f) rank 1.
"""
from dataclasses import dataclass

import torch


@dataclass
class WorldCube:
    scale_factor: torch.Tensor
    shift: torch.Tensor

    def to(self, device):
        return WorldCube(self.scale_factor.to(device), self.shift.to(device))

    def as_dict(self):
        return {"scale_factor": float(self.scale_factor.reshape(-1)[0]), "shift": [float(s) for s in self.shift.cpu()]}


def _frustum_corners(K, H, W, near, far):
    """The 8 homogeneous corners of a camera's view frustum between depths near and far (camera frame:
    x right, y up, looking down -z), ``_get_view_frustum_corners`` (src/common/pose_utils.py:131-149):
    per (left/right, up/down, near/far) corner the image-plane extent (cx / fx, cy / fy, (W - cx) / fx,
    (H - cy) / fy) scaled by the depth, in the reference's order (left before right, up before down,
    near before far)."""
    assert 0 < near < far
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    xs = (-cx / fx, (W - cx) / fx)
    ys = (cy / fy, -(H - cy) / fy)
    rows = [[x * d, y * d, -d, 1.0] for x in xs for y in ys for d in (near, far)]
    return torch.tensor([[float(v) for v in r] for r in rows], dtype=torch.float32)


def compute_world_cube(camera_to_lidar, intrinsic_mats, image_sizes, lidar_poses, ray_range, padding=0.1,
                       traj_bounding_box=None, submap=None):
    """``compute_world_cube`` (src/common/pose_utils.py:222-314), every branch, fp32 torch on the host:
    * poses: the ground-truth lidar poses (N, 4, 4), re-based on the first pose unless ``submap`` is set
      (:244-248), or, without poses, the 8 corners of ``traj_bounding_box`` as identity-rotation poses
      (:228-242);
    * with a camera (``camera_to_lidar`` given, Fusion Portable calibrations): camera poses =
      lidar poses @ camera_to_lidar^-1, and the points are every camera's view-frustum corners between
      the ray range's depths (one K and image size (H, W) for all, or one per pose) plus every camera and
      lidar position (:250-283);
    * without: the (+-max range)^3 cube corners transformed by every lidar pose plus the lidar positions
      (:285-302);
    then origin = the points' box centre, scale = |box diagonal| / (2 sqrt 3) (1 + padding),
    WorldCube(scale, -origin) (:304-314).  Callers pass padding=0.3 (src/loner.py:104,
    examples/fdt_optimize_implicit_map.py:232-233)."""
    assert 0 <= padding < 1
    assert lidar_poses is not None or traj_bounding_box is not None
    if lidar_poses is None:
        xs, ys, zs = traj_bounding_box["x"], traj_bounding_box["y"], traj_bounding_box["z"]
        combos = torch.tensor([[x, y, z] for x in xs for y in ys for z in zs], dtype=torch.float32)
        lidar_poses = torch.eye(4).tile((8, 1, 1))
        lidar_poses[:, :3, 3] = combos
    else:
        lidar_poses = torch.as_tensor(lidar_poses, dtype=torch.float32)
        if submap is None:
            lidar_poses = lidar_poses @ lidar_poses[0].inverse()
    if camera_to_lidar is not None:
        cam_poses = lidar_poses @ torch.as_tensor(camera_to_lidar, dtype=torch.float32).inverse()
        n = cam_poses.shape[0]
        Ks = torch.as_tensor(intrinsic_mats, dtype=torch.float32)
        if Ks.dim() == 2:
            Ks = Ks.expand(n, 3, 3)
        hw = torch.as_tensor(image_sizes, dtype=torch.float32)
        if hw.shape == (2,):
            hw = hw.expand(n, 2)
        assert hw.shape[0] == n
        corners = [(c2w[:3, :] @ _frustum_corners(K, h_w[0], h_w[1], ray_range[0], ray_range[1]).T).T
                   for K, h_w, c2w in zip(Ks, hw, cam_poses)]
        positions = torch.cat([cam_poses[:, :3, 3], lidar_poses[:, :3, 3]], 0)
    else:
        m = float(ray_range[1])
        box = torch.tensor([[-m, -m, -m, 1], [-m, m, -m, 1], [m, -m, -m, 1], [m, m, -m, 1],
                            [-m, -m, m, 1], [-m, m, m, 1], [m, -m, m, 1], [m, m, m, 1]], dtype=torch.float32)
        corners = [(p[:3, :] @ box.T).T for p in lidar_poses]
        positions = lidar_poses[:, :3, 3]
    pts = torch.cat([torch.cat(corners, 0), positions])
    mn, mx = pts.min(0)[0], pts.max(0)[0]
    origin = mn + (mx - mn) / 2
    scale = (torch.linalg.norm(mx - mn) / (2 * torch.sqrt(torch.tensor([3.0])))) * (1 + padding)
    return WorldCube(scale.reshape(1).float(), (-origin).float())


def get_far_val(pts_o, pts_d, no_nan=False):
    if no_nan:
        pts_d = pts_d + 1e-15
    dirs = torch.tensor([[-1.0], [1.0]], device=pts_o.device, dtype=pts_o.dtype)
    t = (dirs[..., None] - pts_o[:, [0, 1, 2]]) / pts_d[:, [0, 1, 2]]
    return t.clamp(min=0).max(dim=0)[0].min(dim=1)[0].unsqueeze(1)


def build_lidar_rays(directions, distances, lidar_pose, ray_range, world_cube, ignore_world_cube=False):
    """directions (3,P) sensor frame, distances (P,), lidar_pose (4,4) -> rays (P',13), depths (P',)."""
    scale = world_cube.scale_factor.to(directions.device)
    depths = distances / scale
    o = (lidar_pose[:3, 3] + world_cube.shift.to(directions.device)) / scale
    o = o.tile(directions.shape[1], 1)
    d = (lidar_pose[:3, :3] @ directions.type(lidar_pose.dtype)).T
    d = d / torch.norm(d, dim=1, keepdim=True)
    if not ignore_world_cube:
        assert (o.abs().max(dim=1)[0] > 1).sum() == 0, "ray origins are outside the world cube"
    near = ray_range[0] / scale * torch.ones_like(o[:, :1])
    far_range = ray_range[1] / scale * torch.ones_like(o[:, :1])
    far = torch.minimum(far_range, get_far_val(o, d, no_nan=True))
    rays = torch.cat([o, d, -d, torch.zeros_like(o[:, :2]), near, far], 1)
    if ignore_world_cube:
        return rays, depths
    valid = (far > (near + 1.0 / scale))[..., 0]
    return rays[valid], depths[valid]


def build_keyframe_rays(scan, lidar_pose, lidar_indices, ray_range, world_cube, sky_indices=None):
    """``KeyFrame.build_lidar_rays``: selected scan rays, then sky rays at distance r_max + 1."""
    rays, depths = build_lidar_rays(scan["directions"][:, lidar_indices], scan["distances"][lidar_indices], lidar_pose,
                                    ray_range, world_cube)
    if sky_indices is not None and scan.get("sky_directions") is not None and scan["sky_directions"].numel() > 0:
        sky_dirs = scan["sky_directions"][:, sky_indices]
        sky_d = torch.full((sky_dirs.shape[1],), float(ray_range[1]) + 1.0, dtype=sky_dirs.dtype, device=sky_dirs.device)
        srays, sdepths = build_lidar_rays(sky_dirs, sky_d, lidar_pose.detach(), ray_range, world_cube)
        rays = torch.cat((rays, srays))
        depths = torch.cat((depths, sdepths))
    return rays, depths


class RayWindow:
    """The active keyframe window, resident on the GPU, from which every optimiser step selects and
    builds its LiDAR rays on the device (``lnr_build_lidar_rays``) instead of on the CPU
    (``Optimizer._do_iterate_optimizer``, src/mapping/optimizer.py:363-424, with
    ``data_prep_on_cpu``).

    ``scans``: one dict per keyframe with ``directions`` (3,P) sensor frame, ``distances`` (P,) metres,
    optional ``sky_directions`` (3,Q) and ``pose`` (4,4) lidar pose (or pass ``poses``).  The
    per-keyframe slot counts follow the reference exactly: MASK takes min(int(0.75 n), #trunk)
    trunk points and min(n - int(0.75 n), #other) others (randperm prefixes), RANDOM takes n, and
    ``n_sky`` sky rays are drawn when the scan has sky directions (optimizer.py:383-386).

    The reference asserts that every ray origin lies inside the world cube (ray_utils.py:301-303)
    and drops rays with far <= near + 1 m / scale (:319-322).  The first is checked here, once per
    window; for the second the window checks once whether ANY point can be invalid (``all_valid``).
    When none can, a step's batch has a fixed size and needs no host synchronisation."""

    def __init__(self, scans, world_cube, ray_range, n_lidar=512, n_sky=0, strategy="RANDOM", poses=None,
                 device="cuda"):
        from . import _lib as L
        if strategy not in ("RANDOM", "MASK"):
            raise ValueError(f"unsupported ray selection strategy {strategy!r} (optimizer.py:363-381)")
        self.device = torch.device(device)
        self.strategy = strategy
        self.n_lidar = int(n_lidar)
        self.n_sky = int(n_sky)
        K = len(scans)
        if K == 0:
            raise ValueError("empty keyframe window")
        poses = torch.stack([s["pose"] for s in scans]) if poses is None else torch.as_tensor(poses)
        poses = poses.detach().to("cpu", torch.float32)
        scale = float(world_cube.scale_factor.reshape(-1)[0])
        shift = [float(v) for v in world_cube.shift.reshape(-1)]
        origins = (poses[:, :3, 3] + world_cube.shift.reshape(1, 3).float()) / world_cube.scale_factor.reshape(1, 1)
        assert (origins.abs().max(dim=1)[0] > 1).sum() == 0, \
            f"{int((origins.abs().max(dim=1)[0] > 1).sum())} ray origins are outside the world cube"
        dirs, dists, order, n_trunk, sky, scan_off, sky_off = [], [], [], [], [], [0], [0]
        n_sel, n_sel_trunk, n_sky_k = [], [], []
        nt_want = int(self.n_lidar * 0.75)
        for s in scans:
            d = s["directions"].detach().to("cpu", torch.float32)
            r = s["distances"].detach().to("cpu", torch.float32).reshape(-1)
            P = r.shape[0]
            if P == 0:
                raise ValueError("a keyframe scan has no points")
            dirs.append(d.T.contiguous())
            dists.append(r)
            scan_off.append(scan_off[-1] + P)
            if strategy == "MASK":
                z = (d * r)[2]  # xyz = ray_directions * distances (optimizer.py:372)
                trunk = (0.5 < z) & (z < 8)
                idx = torch.arange(P, dtype=torch.int32)
                order.append(torch.cat([idx[trunk], idx[~trunk]]))
                nt = int(trunk.sum())
                n_trunk.append(nt)
                ts = min(nt_want, nt)
                n_sel_trunk.append(ts)
                n_sel.append(ts + min(self.n_lidar - nt_want, P - nt))
            else:
                n_sel.append(self.n_lidar)
            sd = s.get("sky_directions")
            q = 0 if sd is None else int(sd.shape[1])
            if q > 0:
                sky.append(sd.detach().to("cpu", torch.float32).T.contiguous())
            sky_off.append(sky_off[-1] + q)
            n_sky_k.append(self.n_sky if (self.n_sky > 0 and q > 0) else 0)
        dev = self.device
        i32 = dict(dtype=torch.int32, device=dev)
        self.poses = poses[:, :3, :4].reshape(K, 12).contiguous().to(dev)
        self.dirs = torch.cat(dirs).contiguous().to(dev)
        self.dists = torch.cat(dists).contiguous().to(dev)
        self.scan_off = torch.tensor(scan_off, **i32)
        self.sky_dirs = torch.cat(sky).contiguous().to(dev) if sky else None
        self.sky_off = torch.tensor(sky_off, **i32)
        self.order = torch.cat(order).contiguous().to(dev) if order else None
        self.n_trunk = torch.tensor(n_trunk, **i32) if order else None
        self.n_sel_trunk = torch.tensor(n_sel_trunk, **i32) if order else None
        self.n_sel = torch.tensor(n_sel, **i32)
        self.n_sel_host = list(n_sel)                                       # LiDAR slots per keyframe
        self.sky_count_host = [sky_off[k + 1] - sky_off[k] for k in range(K)]  # sky directions per keyframe
        counts = [a + b for a, b in zip(n_sel, n_sky_k)]
        self.ray_off_host = [0]
        for c in counts:
            self.ray_off_host.append(self.ray_off_host[-1] + c)
        self.ray_off = torch.tensor(self.ray_off_host, **i32)
        self.n_slots = self.ray_off_host[-1]
        self.n_kf = K
        self.scale = scale
        self.ray_range = (float(ray_range[0]), float(ray_range[1]))
        self._L = L
        self.desc = self._desc(self.ray_off, self.n_sel, shift)
        # every point (and sky direction) once: can any ray of this window fail the 1 m filter?
        all_sel = torch.tensor([scan_off[k + 1] - scan_off[k] for k in range(K)], **i32)
        all_off = torch.tensor([scan_off[k] + sky_off[k] for k in range(K + 1)], **i32)
        d_all = self._desc(all_off, all_sel, shift)
        n_all = scan_off[-1] + sky_off[-1]
        self._desc_all, self.n_all = d_all, n_all
        rays, depth, valid = self.build_all()
        self.all_valid = bool(valid.bool().all())  # the one host synchronisation per window

    def build_all(self):
        """Every scan point (then every sky direction) of every keyframe, in order: the rays of
        ``LidarRayDirections.fetch_chunk_rays`` over whole scans (ray_utils.py:262-267), unfiltered,
        with their validity.  Returns (rays (n_all,13), depth (n_all,), valid (n_all,) uint8)."""
        L, dev, n = self._L, self.device, self.n_all
        rays = torch.empty(n, 13, dtype=torch.float32, device=dev)
        depth = torch.empty(n, dtype=torch.float32, device=dev)
        valid = torch.empty(n, dtype=torch.uint8, device=dev)
        L.call("lnr_build_lidar_rays", L.ctypes.byref(self._desc_all), L.SELECT["ALL"], None, 0, 0, n, rays, depth,
               valid, None, None, L.stream(dev))
        return rays, depth, valid

    def _desc(self, ray_off, n_sel, shift):
        L = self._L
        d = L.RayWindowDesc()
        d.n_kf = self.n_kf
        d.scale = self.scale
        for i in range(3):
            d.shift[i] = shift[i]
        d.r_min, d.r_max = self.ray_range
        p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        d.poses, d.dirs, d.dists, d.scan_off = p(self.poses), p(self.dirs), p(self.dists), p(self.scan_off)
        d.order, d.n_trunk, d.n_sel_trunk = p(self.order), p(self.n_trunk), p(self.n_sel_trunk)
        d.sky_dirs, d.sky_off = p(self.sky_dirs), p(self.sky_off)
        d.ray_off, d.n_sel = p(ray_off), p(n_sel)
        d._keep = (ray_off, n_sel)
        return d

    def build(self, key, slot0=0, n=None, rays=None, depth=None, valid=None, point_index=None, far_ref=None,
              given=None, dev_step=None):
        """Enqueue the build of slots [slot0, slot0 + n) for the step keyed by ``key``
        (``lnr_step_key``).  Returns (rays, depth, valid, point_index, far_ref) device tensors; outputs
        may be passed in (preallocated).  ``given``: int32 scan-local indices per slot (parity tests).
        ``dev_step``: a device ``lnr_step_scalars`` whose key is used instead of ``key`` (graph replay)."""
        L = self._L
        n = self.n_slots - slot0 if n is None else n
        dev = self.device
        rays = torch.empty(n, 13, dtype=torch.float32, device=dev) if rays is None else rays
        depth = torch.empty(n, dtype=torch.float32, device=dev) if depth is None else depth
        valid = torch.empty(n, dtype=torch.uint8, device=dev) if valid is None else valid
        far_ref = torch.empty(1, dtype=torch.float32, device=dev) if far_ref is None else far_ref
        sel = L.SELECT["GIVEN"] if given is not None else L.SELECT[self.strategy]
        desc = self.desc
        if dev_step is not None:
            desc = L.RayWindowDesc.from_buffer_copy(self.desc)
            desc.dev_step = dev_step.data_ptr()
        L.call("lnr_build_lidar_rays", L.ctypes.byref(desc), sel, given, int(key) & 0xFFFFFFFF, slot0, n, rays,
               depth, valid, point_index, far_ref, L.stream(dev))
        return rays, depth, valid, point_index, far_ref
