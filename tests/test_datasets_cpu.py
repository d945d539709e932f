"""NeRF-synthetic ingest (datasets/nerf.py, color_utils.py, ray_utils.py of the
reference): PNG decoding (all five scanline filters),
alpha blending onto white, cv2-style linear resize, pose conversion to
[right down front] at radius 1.5, intrinsics from camera_angle_x."""
import json
import math
import struct
import zlib

import numpy as np
import torch

import synthetic as S
from datasets import NeRFDataset, dataset_dict
from datasets.png import read_png, write_png
from datasets.ray_utils import get_ray_directions, get_rays


def _png_with_filters(path, img):
    """Encoder using filter type (row % 5) so the decoder sees every filter."""
    H, W, C = img.shape
    rows, prev = [], np.zeros(W * C, np.int32)
    for y in range(H):
        cur = img[y].reshape(-1).astype(np.int32)
        ft = y % 5
        left = np.concatenate([np.zeros(C, np.int32), cur[:-C]])
        ul = np.concatenate([np.zeros(C, np.int32), prev[:-C]])
        if ft == 0:
            f = cur
        elif ft == 1:
            f = cur - left
        elif ft == 2:
            f = cur - prev
        elif ft == 3:
            f = cur - (left + prev) // 2
        else:
            p = left + prev - ul
            pa, pb, pc = abs(p - left), abs(p - prev), abs(p - ul)
            f = cur - np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, prev, ul))
        rows.append(bytes([ft]) + (f & 255).astype(np.uint8).tobytes())
        prev = cur

    def chunk(kind, body):
        return struct.pack(">I", len(body)) + kind + body + struct.pack(">I", zlib.crc32(kind + body) & 0xffffffff)

    ctype = {3: 2, 4: 6}[C]
    with open(path, "wb") as fh:
        fh.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", W, H, 8, ctype, 0, 0, 0)) +
                 chunk(b"IDAT", zlib.compress(b"".join(rows))) + chunk(b"IEND", b""))


def test_png_decoder_all_filters(tmp_path):
    rng = np.random.default_rng(0)
    for C in (3, 4):
        img = rng.integers(0, 256, (13, 11, C), dtype=np.uint8)
        _png_with_filters(str(tmp_path / "f.png"), img)
        assert np.array_equal(read_png(str(tmp_path / "f.png")), img)
        write_png(str(tmp_path / "p.png"), img)
        assert np.array_equal(read_png(str(tmp_path / "p.png")), img)


def test_ray_directions_match_the_bench_camera():
    K = S.intrinsics(64, 48)
    assert torch.equal(get_ray_directions(48, 64, K), S.get_ray_directions(48, 64, K))
    d = get_ray_directions(4, 4, K)
    c2w = torch.eye(4)[:3]
    o, r = get_rays(d, c2w)
    assert torch.equal(r, d) and torch.equal(o, torch.zeros_like(d))


def test_nerf_synthetic_loader(tmp_path):
    angle = 0.6911112070083618  # Lego
    rng = np.random.default_rng(1)
    frames, imgs = [], []
    for i in range(3):
        th = 2 * math.pi * i / 3
        c2w = np.eye(4)
        c2w[:3, 3] = [4.0 * math.cos(th), 4.0 * math.sin(th), 1.0]  # blender units, radius != 1.5
        frames.append({"file_path": f"./train/r_{i}", "transform_matrix": c2w.tolist()})
        img = rng.integers(0, 256, (16, 16, 4), dtype=np.uint8)
        (tmp_path / "train").mkdir(exist_ok=True)
        write_png(str(tmp_path / "train" / f"r_{i}.png"), img)
        imgs.append(img)
    json.dump({"camera_angle_x": angle, "frames": frames}, open(tmp_path / "transforms_train.json", "w"))
    ds = NeRFDataset(str(tmp_path), split='train', downsample=0.01)
    assert ds.img_wh == (8, 8)
    fx = 0.5 * 800 / np.tan(0.5 * angle) * 0.01
    assert abs(float(ds.K[0, 0]) - fx) < 1e-4 and float(ds.K[0, 2]) == 4.0
    assert ds.poses.shape == (3, 3, 4) and ds.rays.shape == (3, 64, 3)
    # [right up back] -> [right down front], camera centre at radius 1.5
    assert torch.allclose(ds.poses[:, :, 3].norm(dim=1), torch.full((3,), 1.5), atol=1e-5)
    assert float(ds.poses[0, 1, 1]) == -1.0 and float(ds.poses[0, 2, 2]) == -1.0
    # alpha blended onto white, then 16 -> 8 linear resize = 2x2 mean
    f = imgs[0].astype(np.float32) / 255
    rgb = f[..., :3] * f[..., 3:] + (1 - f[..., 3:])
    want = rgb.reshape(8, 2, 8, 2, 3).mean((1, 3)).reshape(-1, 3)
    np.testing.assert_allclose(ds.rays[0].numpy(), want, atol=1e-6)
    assert ds.gt_u8().dtype == torch.uint8
    try:
        dataset_dict['rtmv']('x')
        raise AssertionError("expected NotImplementedError")
    except NotImplementedError:
        pass


def test_nsvf_synthetic_loader(tmp_path):
    root = tmp_path / "Synthetic_NeRF" / "Lego"
    (root / "rgb").mkdir(parents=True)
    (root / "pose").mkdir()
    (root / "intrinsics.txt").write_text("1111.1110311937682 0. 0. 0.\n0. 1111.1110311937682 0. 0.\n")
    (root / "bbox.txt").write_text("-0.6 -1.1 -0.4 0.6 1.1 1.0 0.1\n")
    rng = np.random.default_rng(2)
    for split, n in (("0", 2), ("1", 1), ("2", 1)):
        for i in range(n):
            c2w = np.eye(4)
            c2w[:3, 3] = rng.uniform(-3, 3, 3)
            np.savetxt(root / "pose" / f"{split}_{i:04d}.txt", c2w)
            write_png(str(root / "rgb" / f"{split}_{i:04d}.png"), rng.integers(0, 256, (8, 8, 4), dtype=np.uint8))
    ds = dataset_dict['nsvf'](str(root), split='train', downsample=0.01)
    assert ds.img_wh == (8, 8) and abs(float(ds.K[0, 0]) - 11.111110311937682) < 1e-5
    shift = np.array([0.0, 0.0, 0.3])
    scale = 1.1 * 1.05 * 2.2 / 2  # largest side 2.2, x1.05, x1.1 for Lego
    assert np.allclose(ds.shift, shift) and abs(ds.scale - scale) < 1e-9
    raw = np.loadtxt(root / "pose" / "0_0000.txt")[:3]
    want = (raw[:, 3] - shift) / (2 * scale)
    assert np.allclose(ds.poses[0, :, 3].numpy(), want, atol=1e-6)
    assert ds.rays.shape == (2, 64, 3)
    assert dataset_dict['nsvf'](str(root), split='test', downsample=0.01).poses.shape == (1, 3, 4)


def test_colmap_model_and_loader(tmp_path):
    from PIL import Image as PILImage

    from datasets import colmap_utils as CU
    from datasets.ray_utils import center_poses
    root = tmp_path / "garden"
    (root / "sparse" / "0").mkdir(parents=True)
    (root / "images").mkdir()
    rng = np.random.default_rng(3)
    cams = {1: CU.Camera(1, "PINHOLE", 16, 12, np.array([20.0, 21.0, 8.0, 6.0]))}
    ims = {}
    for i in range(9):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        name = f"img_{8 - i:03d}.jpg"  # ids and names in opposite orders: poses are sorted by name
        ims[i + 1] = CU.Image(i + 1, q, rng.normal(size=3) * 3, 1, name, np.zeros((0, 2)), np.zeros(0, np.int64))
        PILImage.fromarray(rng.integers(0, 256, (12, 16, 3), dtype=np.uint8)).save(root / "images" / name, quality=95)
    pts = {k: CU.Point3D(k, rng.normal(size=3), np.array([1, 2, 3]), 0.5, np.zeros(0), np.zeros(0)) for k in range(20)}
    CU.write_model_binary(str(root / "sparse" / "0"), cams, ims, pts)
    # readers round-trip the model
    rc = CU.read_cameras_binary(str(root / "sparse/0/cameras.bin"))
    ri = CU.read_images_binary(str(root / "sparse/0/images.bin"))
    assert rc[1].model == "PINHOLE" and np.array_equal(rc[1].params, cams[1].params)
    assert ri[3].name == ims[3].name and np.array_equal(ri[3].qvec, ims[3].qvec)
    R = ri[3].qvec2rotmat()
    assert np.allclose(R @ R.T, np.eye(3)) and abs(np.linalg.det(R) - 1) < 1e-9
    ds = dataset_dict['colmap'](str(root), split='train')
    assert ds.img_wh == (16, 12) and float(ds.K[0, 0]) == 20.0 and float(ds.K[1, 2]) == 6.0
    assert ds.poses.shape == (7, 3, 4) and ds.rays.shape == (7, 192, 3)  # images 0 and 8 (i % 8 == 0) are test
    # expected poses: c2w sorted by name, centred on the point cloud, closest camera at distance 1
    order = sorted(ims, key=lambda k: ims[k].name)
    c2w = []
    for k in order:
        w2c = np.eye(4)
        w2c[:3, :3], w2c[:3, 3] = CU.qvec2rotmat(ims[k].qvec), ims[k].tvec
        c2w.append(np.linalg.inv(w2c)[:3])
    pc, _, _ = center_poses(np.stack(c2w), np.stack([p.xyz for p in pts.values()]))
    pc[..., 3] /= np.linalg.norm(pc[..., 3], axis=-1).min()
    np.testing.assert_allclose(ds.poses.numpy(), pc[[i for i in range(9) if i % 8 != 0]].astype(np.float32),
                               rtol=1e-5, atol=1e-5)
    assert dataset_dict["colmap"](str(root), split="test").poses.shape == (2, 3, 4)
