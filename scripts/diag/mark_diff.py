"""mark_invisible_cells (networks.py:209-250) on the GPU vs the CPU: how many
cells differ and how close their projections sit to an image border / the
near plane (float64 recomputation)."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "ar-nerf_amd")]
import torch
import synthetic as S
import vren

NEAR = 0.01


def mark(K, poses, W, H, G, scale, c, dev, chunk=64 ** 3):
    ax = torch.arange(G, dtype=torch.int32)
    coords = torch.stack(torch.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3).to(dev)
    K, poses = K.to(dev), poses.to(dev)
    w2c_R = poses[:, :3, :3].transpose(1, 2)
    w2c_T = -w2c_R @ poses[:, :3, 3:]
    out = torch.zeros(G ** 3, device=dev)
    for i in range(0, G ** 3, chunk):
        xyzs = coords[i:i + chunk] / (G - 1) * 2 - 1
        s = min(2 ** (c - 1), scale)
        hgs = s / G
        xyzs_w = (xyzs * (s - hgs)).T
        xyzs_c = w2c_R @ xyzs_w + w2c_T
        uvd = K @ xyzs_c
        uv = uvd[:, :2] / uvd[:, 2:]
        in_image = (uvd[:, 2] >= 0) & (uv[:, 0] >= 0) & (uv[:, 0] < W) & (uv[:, 1] >= 0) & (uv[:, 1] < H)
        cov = (uvd[:, 2] >= NEAR) & in_image
        out[i:i + chunk] = cov.sum(0) / poses.shape[0]
    return out.cpu(), coords.cpu()


for scale in (0.5, 16.0):
    sc = S.AnalyticScene(W=64, H=48, n_images=10, scale=scale)
    C = max(1 + int(torch.ceil(torch.log2(torch.tensor(2 * scale)))), 1)
    for c in range(C):
        a, coords = mark(sc.K, sc.poses, 64, 48, 128, scale, c, "cuda")
        b, _ = mark(sc.K, sc.poses, 64, 48, 128, scale, c, "cpu")
        d = (a != b).nonzero()[:, 0]
        msg = f"scale {scale} cascade {c}: {d.numel()} cells differ"
        if d.numel():
            s = min(2 ** (c - 1), scale); hgs = s / 128
            x = ((coords[d].double() / 127 * 2 - 1) * (s - hgs))
            P = sc.poses.double()
            R = P[:, :3, :3].transpose(1, 2); T = -R @ P[:, :3, 3:]
            xc = R @ x.T + T
            uvd = sc.K.double() @ xc
            uv = uvd[:, :2] / uvd[:, 2:]
            dist = torch.stack([uv[:, 0].abs(), (uv[:, 0] - 64).abs(), uv[:, 1].abs(), (uv[:, 1] - 48).abs()], 0).amin(0)
            dn = (uvd[:, 2] - NEAR).abs()
            md = torch.minimum(dist / 64, dn).amin(0)
            msg += f"; min over cams of relative border/near distance: max {float(md.max()):.3e}"
        print(msg, flush=True)
