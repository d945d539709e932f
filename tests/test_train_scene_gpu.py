"""End to end on the data-ingest path: an NSVF-format scene on disk (PNG
images + pose/intrinsics/bbox text files, rendered from the analytic
synthetic scene) -> datasets.NSVFDataset -> NGPTrainer (mark_invisible_cells,
device-drawn batches, graph replays) -> test PSNR on the held-out split
(scripts/train_scene.py, the reference's train.py flow)."""
import importlib.util
import os

import numpy as np
import pytest
import torch

import synthetic as S
from datasets.png import write_png

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write_scene(root, res=100, n_train=24, n_test=2):
    (root / "rgb").mkdir(parents=True)
    (root / "pose").mkdir()
    fx = 0.5 * 800 / np.tan(0.5 * 0.6911112070083618)
    (root / "intrinsics.txt").write_text(f"{fx} 0. 0. 0.\n")
    b = 0.5 / 1.05  # NSVF scale = 1.05 * half side = 0.5, shift 0: poses unchanged
    (root / "bbox.txt").write_text(f"{-b} {-b} {-b} {b} {b} {b} 0.01\n")
    sc = S.AnalyticScene(W=res, H=res, n_images=n_train + n_test, seed=7)
    for i in range(n_train + n_test):
        split = "0" if i < n_train else "2"
        P = sc.poses[i]
        d = sc.directions @ P[:, :3].t()
        o = P[:, 3].expand_as(d)
        rgb = sc.gt_rgb_rays(o.contiguous(), d.contiguous()).reshape(res, res, 3)
        write_png(str(root / "rgb" / f"{split}_{i:04d}.png"), (rgb.clamp(0, 1) * 255 + 0.5).to(torch.uint8).numpy())
        c2w = np.eye(4)
        c2w[:3] = P.numpy()
        np.savetxt(root / "pose" / f"{split}_{i:04d}.txt", c2w)


def test_nsvf_scene_trains_to_a_useful_psnr(tmp_path):
    root = tmp_path / "Synthetic_Test" / "Sphere"
    _write_scene(root)
    spec = importlib.util.spec_from_file_location("train_scene", os.path.join(ROOT, "scripts", "train_scene.py"))
    ts = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ts)
    res = ts.main(["--dataset", "nsvf", "--root", str(root), "--downsample", "0.125", "--steps", "1500"])
    assert res["test_views"] == 2
    assert res["test_psnr"] > 22.0, res
