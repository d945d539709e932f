"""datasets/ray_utils.py:7-214 of the reference (kornia-free)."""
import numpy as np
import torch


def get_ray_directions(H, W, K, device='cpu', random=False, return_uv=False, flatten=True):
    """Camera-space directions [right down front] through each pixel centre
    (or a random point inside it): ((u - cx + 0.5)/fx, (v - cy + 0.5)/fy, 1)."""
    v, u = torch.meshgrid(torch.arange(H, dtype=torch.float32, device=device),
                          torch.arange(W, dtype=torch.float32, device=device), indexing="ij")
    K = torch.as_tensor(K, dtype=torch.float32)
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    if random:
        d = torch.stack([(u - cx + torch.rand_like(u)) / fx, (v - cy + torch.rand_like(v)) / fy,
                         torch.ones_like(u)], -1)
    else:
        d = torch.stack([(u - cx + 0.5) / fx, (v - cy + 0.5) / fy, torch.ones_like(u)], -1)
    grid = torch.stack([u, v], -1)
    if flatten:
        d, grid = d.reshape(-1, 3), grid.reshape(-1, 2)
    return (d, grid) if return_uv else d


def get_rays(directions, c2w):
    """World-space rays: rays_d = R @ dir (not normalised), rays_o = c2w[..., 3]."""
    if c2w.ndim == 2:
        rays_d = directions @ c2w[:, :3].T
    else:
        # per-ray poses (the training batch, train.py:85-87): d_a = sum_c dir_c R[a][c] c-major, one
        # rounding per op -- the arithmetic of the device batch draw (ngp_sample_batch); a batched
        # 3x3 GEMM here cost ~70 us per 8192-ray batch
        R = c2w[..., :3]
        rays_d = directions[:, None, 0] * R[..., 0] + directions[:, None, 1] * R[..., 1]
        rays_d = rays_d + directions[:, None, 2] * R[..., 2]
    rays_o = c2w[..., 3].expand_as(rays_d)
    return rays_o, rays_d


def normalize(v):
    return v / np.linalg.norm(v)


def average_poses(poses, pts3d=None):
    """ray_utils.py:108-147: centre = mean of the point cloud (or of the
    cameras), z = mean z axis, x = y' x z, y = z x x."""
    center = pts3d.mean(0) if pts3d is not None else poses[..., 3].mean(0)
    z = normalize(poses[..., 2].mean(0))
    y_ = poses[..., 1].mean(0)
    x = normalize(np.cross(y_, z))
    y = np.cross(z, x)
    return np.stack([x, y, z, center], 1)


def center_poses(poses, pts3d=None):
    """ray_utils.py:150-178: poses (and points) in the average pose's frame."""
    pose_avg = average_poses(poses, pts3d)
    pose_avg_homo = np.eye(4)
    pose_avg_homo[:3] = pose_avg
    pose_avg_inv = np.linalg.inv(pose_avg_homo)
    last_row = np.tile(np.array([0, 0, 0, 1]), (len(poses), 1, 1))
    poses_centered = (pose_avg_inv @ np.concatenate([poses, last_row], 1))[:, :3]
    if pts3d is not None:
        return poses_centered, pts3d @ pose_avg_inv[:, :3].T + pose_avg_inv[:, 3:].T, pose_avg
    return poses_centered, pose_avg


def create_spheric_poses(radius, mean_h, n_poses=120):
    """ray_utils.py:180-216: a circle of n_poses cameras around the z axis."""
    def spheric_pose(theta, phi, radius):
        trans_t = np.array([[1, 0, 0, 0], [0, 1, 0, 2 * mean_h], [0, 0, 1, -radius]])
        rot_phi = np.array([[1, 0, 0], [0, np.cos(phi), -np.sin(phi)], [0, np.sin(phi), np.cos(phi)]])
        rot_theta = np.array([[np.cos(theta), 0, -np.sin(theta)], [0, 1, 0], [np.sin(theta), 0, np.cos(theta)]])
        c2w = rot_theta @ rot_phi @ trans_t
        return np.array([[-1, 0, 0], [0, 0, 1], [0, 1, 0]]) @ c2w
    return np.stack([spheric_pose(th, -np.pi / 12, radius) for th in np.linspace(0, 2 * np.pi, n_poses + 1)[:-1]], 0)
