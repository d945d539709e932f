"""End to end on the data-ingest path: an NSVF-format scene on disk (PNG
images + pose/intrinsics/bbox text files, rendered from the analytic
synthetic scene) -> datasets.NSVFDataset -> NGPTrainer (mark_invisible_cells,
device-drawn batches, graph replays) -> test PSNR on the held-out split
(scripts/train_scene.py, the reference's train.py flow)."""
import importlib.util
import os

import pytest

import synthetic as S

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_nsvf_scene_trains_to_a_useful_psnr(tmp_path):
    root = tmp_path / "Synthetic_Test" / "Sphere"
    S.write_nsvf_scene(str(root), res=100, n_train=24, n_test=2)
    spec = importlib.util.spec_from_file_location("train_scene", os.path.join(ROOT, "scripts", "train_scene.py"))
    ts = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ts)
    res = ts.main(["--dataset", "nsvf", "--root", str(root), "--downsample", "0.125", "--steps", "1500"])
    assert res["test_views"] == 2
    assert res["test_psnr"] > 22.0, res
