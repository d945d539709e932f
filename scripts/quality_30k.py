#!/usr/bin/env python3
"""Quality after the reference schedule (SURVEY.md §0 / north_star "PSNR
within 0.2 dB of reference after 30k steps"): the analytic scene written as
an NSVF-format dataset (synthetic.write_nsvf_scene) -> scripts/train_scene.py
(train.py's flow: mark_invisible_cells, 8192-ray batches, occupancy updates
every 16 steps with 256 warm-up steps, Adam lr 1e-2 cosine-annealed per
epoch to lr/30 over 30 epochs x 1000 steps, the 'raw' loss) -> mean test
PSNR, twice: the product defaults (chunked field evaluation, binned
fine-level hash backward) and the exact mode (every marched sample through
the field, per-sample atomic hash backward).  The reference itself cannot
run here (CUDA), so "reference" = the exact mode of the same kernels.
Prints one JSON line."""
import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd")]


def _train(args):
    """scripts/train_scene.py in a child process of its own (one trainer per
    process, as in training; the GPU state of one run cannot touch the next)"""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "train_scene.py")] + args,
                         check=True, stdout=subprocess.PIPE, text=True).stdout
    r = json.loads(out.strip().splitlines()[-1])
    print(f"[quality_30k] {' '.join(args[-3:])}: {json.dumps(r)[:200]}", file=sys.stderr, flush=True)  # (progress)
    return r


def run(steps=30000, res=400, n_train=100, n_test=10, seed=4, root=None):
    import synthetic as S
    with tempfile.TemporaryDirectory() as tmp:
        scene = root or os.path.join(tmp, "Synthetic_NeRF", "Analytic")
        if root is None:
            S.write_nsvf_scene(scene, res=res, n_train=n_train, n_test=n_test)
        args = ["--dataset", "nsvf", "--root", scene, "--downsample", str(res / 800), "--steps", str(steps),
                "--seed", str(seed)]
        default = _train(args)
        exact = _train(args + ["--exact"])
    return {"steps": steps, "schedule": "30 epochs x 1000 steps (scaled to steps), lr 1e-2 cosine to lr/30, raw loss",
            "scene": f"analytic sphere+box as NSVF, {n_train} train / {n_test} test views at {res}x{res}",
            "psnr_default": default["test_psnr"], "psnr_exact": exact["test_psnr"],
            "delta_db": round(default["test_psnr"] - exact["test_psnr"], 3),
            "train_rays_per_s_default": default["train_rays_per_s"],
            "train_rays_per_s_exact": exact["train_rays_per_s"]}


def run_seeds(seeds, steps=30000, res=400):
    """run() for several seeds (model init, batches, occupancy draws) on one written scene: per-seed PSNRs
    of both modes, their means and the mean / spread of the per-seed difference."""
    import synthetic as S
    with tempfile.TemporaryDirectory() as tmp:
        scene = os.path.join(tmp, "Synthetic_NeRF", "Analytic")
        S.write_nsvf_scene(scene, res=res, n_train=100, n_test=10)
        per = [run(steps, res, seed=sd, root=scene) for sd in seeds]
    d = [p["delta_db"] for p in per]
    mean = lambda v: round(sum(v) / len(v), 3)  # noqa: E731
    return {"steps": steps, "seeds": list(seeds), "psnr_default": [p["psnr_default"] for p in per],
            "psnr_exact": [p["psnr_exact"] for p in per], "mean_default": mean([p["psnr_default"] for p in per]),
            "mean_exact": mean([p["psnr_exact"] for p in per]), "delta_db": d, "mean_delta_db": mean(d),
            "delta_range_db": [min(d), max(d)], "scene": per[0]["scene"]}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30000)
    ap.add_argument("--res", type=int, default=400)
    ap.add_argument("--root", default=None, help="an existing NSVF scene instead of the synthetic one")
    ap.add_argument("--seeds", default=None, help="comma-separated seeds: run_seeds (both modes per seed)")
    a = ap.parse_args()
    if a.seeds:
        print(json.dumps(run_seeds([int(x) for x in a.seeds.split(",")], a.steps, a.res)))
    else:
        print(json.dumps(run(a.steps, a.res, root=a.root)))
