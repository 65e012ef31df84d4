"""World cube and LiDAR ray construction (host-side data preparation feeding the hot path).

Mirrors the reference's interface and semantics:
  WorldCube                ``src/common/pose_utils.py:23-57``
  compute_world_cube       ``src/common/pose_utils.py:222-314`` (lidar-only, trajectory or bbox)
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


def compute_world_cube(lidar_poses=None, ray_range=(1.0, 75.0), padding=0.3, traj_bounding_box=None):
    """Lidar-only ``compute_world_cube``; callers in the reference pass padding=0.3
    (src/loner.py:104, examples/fdt_optimize_implicit_map.py:232)."""
    assert 0 <= padding < 1
    if lidar_poses is None:
        xs, ys, zs = traj_bounding_box["x"], traj_bounding_box["y"], traj_bounding_box["z"]
        combos = torch.tensor([[x, y, z] for x in xs for y in ys for z in zs], dtype=torch.float32)
        lidar_poses = torch.eye(4).tile((8, 1, 1))
        lidar_poses[:, :3, 3] = combos
    else:
        lidar_poses = lidar_poses @ lidar_poses[0].inverse()
    m = float(ray_range[1])
    corners = torch.tensor([[-m, -m, -m, 1], [-m, m, -m, 1], [m, -m, -m, 1], [m, m, -m, 1],
                            [-m, -m, m, 1], [-m, m, m, 1], [m, -m, m, 1], [m, m, m, 1]], dtype=lidar_poses.dtype)
    all_corners = torch.cat([(p[:3, :] @ corners.T).T for p in lidar_poses], 0)
    pts = torch.cat([all_corners, lidar_poses[:, :3, 3]])
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
