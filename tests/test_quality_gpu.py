"""Training quality against fp32-oracle trajectories (north_star "PSNR within
0.2 dB of reference"; train.py:242-245, README.md:116-121).

tests/golden/make_quality.py runs the reference's own training-loop glue on
the CPU oracle (fp32 autograd; 2000 steps of 2048 rays, 20 epochs x 100 steps
of the cosine schedule, occupancy updates every 16 steps, the analytic scene
at 100x100) and stores the held-out test PSNR.  The product trains the same
problem -- same scene, init, lr schedule and batches (image / pixel indices
and march noise of every step, drawn on the host and given to step()) -- on
the device.  Occupancy cells are drawn by each side's own RNG (same
distribution), so trajectories are compared through the PSNR.

The fixtures, which differ in the precision at the tcnn-module boundary:
  * quality_oracle.json (+ _occ1 / _occ2: other occupancy draws) -- the
    reference's precision: the tcnn modules return fp16, as tinycudann's do,
    so the gradients the glue hands back into them (dL/dh from TruncExp's
    backward, dL/drgb) are rounded to fp16 -- at the loss scale of the
    GradScaler that Lightning's precision=16 attaches (train.py:291: init
    2^16, x0.5 and a skipped step on inf / nan, x2 after 2000 clean steps),
    as on the GPU; the gradients are unscaled in fp32 before Adam;
  * quality_oracle_f32out.json -- the same glue with that boundary in fp32
    (no rounding there at all).
The bar: the product within 0.2 dB of the reference-precision runs (the
range of the three occupancy draws, widened by 0.2 dB on each side)."""
import json
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLD)

BAR_DB = 0.2  # north_star: PSNR within 0.2 dB of the reference


def _fx(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


@pytest.mark.parametrize("mode", ["default", "exact"])
def test_test_psnr_against_the_reference_precision_oracle_runs(mode):
    """default: the product path (chunked field evaluation, hybrid hash
    backward); exact: every marched sample through the field, per-sample
    atomic hash backward.  Both take fp16 MFMA operands in the MLP forward
    and backward, weight gradients included (tcnn's precision)."""
    import make_quality as MQ
    refs = [_fx(n) for n in ("quality_oracle.json", "quality_oracle_occ1.json", "quality_oracle_occ2.json")]
    assert all(r.get("grad_scaler") for r in refs), "the reference-precision fixtures model the AMP GradScaler"
    ref_prec = [r["test_psnr"] for r in refs]
    f32_prec = _fx("quality_oracle_f32out.json")["test_psnr"]
    kw = {} if mode == "default" else dict(chunk_first=0, hash_backward="atomic")
    res = MQ.product_run("cuda", **kw)
    p = res["test_psnr"]
    print(f"[{mode}] product test PSNR {p:.3f} dB (views {res['test_psnr_views']}); fp32 oracle at the reference's "
          f"precision (fp16 tcnn boundary under the GradScaler) {min(ref_prec):.3f}-{max(ref_prec):.3f} dB "
          f"({p - sum(ref_prec) / len(ref_prec):+.3f} vs their mean); fp32 boundary {f32_prec:.3f} dB "
          f"({p - f32_prec:+.3f}); final loss {res['final_loss_mean_last_100']:.3e}; {res['steps']} steps in "
          f"{res['train_wall_s']} s")
    assert torch.isfinite(torch.tensor(res["loss_curve_every_50"])).all()
    assert min(ref_prec) - BAR_DB <= p <= max(ref_prec) + BAR_DB, (p, ref_prec)
