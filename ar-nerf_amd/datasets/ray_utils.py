"""datasets/ray_utils.py:7-70 of the reference (kornia-free)."""
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
        rays_d = torch.einsum('nc,nac->na', directions, c2w[..., :3])
    rays_o = c2w[..., 3].expand_as(rays_d)
    return rays_o, rays_d
