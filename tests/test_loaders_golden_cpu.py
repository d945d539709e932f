"""The dataset loaders (ar-nerf_amd/datasets: NSVFDataset, NeRFDataset,
ColmapDataset) against fixtures from the REFERENCE's own loaders
(datasets/nsvf.py:13-100, datasets/nerf.py:13-100, datasets/colmap.py:15-166
with colmap_utils.py's binary readers, ray_utils.get_ray_directions /
center_poses / create_spheric_poses and color_utils.read_image), run on the
same synthetic scenes
(tests/golden/make_loaders.py: RGBA frames -> the alpha blend onto white, an
off-centre NSVF bbox -> pose shift and scale, Blender [right up back]
matrices at radius 4 -> the flip and the rescale to 1.5; a COLMAP model
with a PINHOLE camera, image ids out of name order, a rotated / shifted /
scaled world and RGBA frames -> the name sort, center_poses, the
min-distance rescale, the every-8th test split, rgb x alpha).  Intrinsics,
image size, poses and ray directions equal the reference's to fp32
rounding; the blended pixels bit for bit."""
import hashlib
import os
import sys
import tempfile

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))


@pytest.fixture(scope="module")
def scenes():
    import make_loaders as ML
    with tempfile.TemporaryDirectory() as tmp:
        yield ML, ML.write_scenes(tmp) + (ML.write_colmap_scene(tmp),)


@pytest.mark.parametrize("kind", ["nsvf", "nerf"])
@pytest.mark.parametrize("split", ["train", "test"])
def test_loader_matches_reference_loader(scenes, kind, split):
    from datasets import NeRFDataset, NSVFDataset
    ML, (nsvf_root, nerf_root, _) = scenes
    fx = np.load(os.path.join(HERE, "golden", "loaders.npz"))
    cls, root = (NSVFDataset, nsvf_root) if kind == "nsvf" else (NeRFDataset, nerf_root)
    ds = cls(root, split=split, downsample=ML.RES / 800)
    p = f"{kind}_{split}_"
    assert np.array_equal(ds.K.numpy(), fx[p + "K"])
    assert tuple(ds.img_wh) == tuple(fx[p + "img_wh"])
    np.testing.assert_allclose(ds.poses.numpy(), fx[p + "poses"], rtol=0, atol=2e-7)
    np.testing.assert_allclose(ds.directions.numpy(), fx[p + "directions"], rtol=0, atol=1e-7)
    rays = ds.rays.numpy() if hasattr(ds.rays, "numpy") else np.asarray(ds.rays)
    assert tuple(rays.shape) == tuple(fx[p + "rays_shape"])
    assert np.array_equal(rays[:, ::53], fx[p + "rays_sub"])
    assert hashlib.sha256(np.ascontiguousarray(rays.astype(np.float32)).tobytes()).hexdigest() == str(fx[p + "rays_sha"])
    if kind == "nsvf":
        np.testing.assert_allclose(np.asarray(ds.shift), fx["nsvf_shift"], rtol=0, atol=1e-12)
        assert abs(float(ds.scale) - float(fx["nsvf_scale"])) <= 1e-12


@pytest.mark.parametrize("split", ["train", "test", "test_traj"])
def test_colmap_loader_matches_reference_loader(scenes, split):
    from datasets import ColmapDataset
    ML, (_, _, colmap_root) = scenes
    fx = np.load(os.path.join(HERE, "golden", "loaders.npz"))
    ds = ColmapDataset(colmap_root, split=split)
    if split == "test_traj":  # create_spheric_poses(1.2, mean camera height) (ray_utils.py:180-205)
        np.testing.assert_allclose(ds.poses.numpy(), fx["colmap_test_traj_poses"], rtol=0, atol=2e-7)
        return
    p = f"colmap_{split}_"
    assert np.array_equal(ds.K.numpy(), fx[p + "K"])
    assert tuple(ds.img_wh) == tuple(fx[p + "img_wh"])
    np.testing.assert_allclose(ds.poses.numpy(), fx[p + "poses"], rtol=0, atol=2e-7)
    np.testing.assert_allclose(ds.directions.numpy(), fx[p + "directions"], rtol=0, atol=1e-7)
    np.testing.assert_allclose(np.asarray(ds.pts3d), fx[p + "pts3d"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(np.asarray(ds.blender_trans), fx[p + "blender_trans"], rtol=0, atol=1e-12)
    assert abs(float(ds.blender_scale) - float(fx[p + "blender_scale"])) <= 1e-12
    rays = ds.rays.numpy() if hasattr(ds.rays, "numpy") else np.asarray(ds.rays)
    assert tuple(rays.shape) == tuple(fx[p + "rays_shape"])
    assert np.array_equal(rays[:, ::53], fx[p + "rays_sub"])
    assert hashlib.sha256(np.ascontiguousarray(rays.astype(np.float32)).tobytes()).hexdigest() == str(fx[p + "rays_sha"])
