#!/usr/bin/env python3
"""Train the product on the oracle-fixture problem (tests/golden/make_quality.py
product_run, default mode) and save what the test render reads -- fp32
parameters, density grid, bitfield -- plus the per-step losses, so the same
trained state can be rendered through the reference's glue on the CPU oracle
(scripts/quality_glue_render.py): separates a training difference from a
rendering difference in the product-vs-oracle PSNR comparison.
usage: quality_state.py OUT_DIR"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "ar-nerf_amd")]
import torch  # noqa: E402

import make_quality as MQ  # noqa: E402


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    import trainer
    keep = {}
    orig = trainer.NGPTrainer.__init__

    def init(self, *a, **k):
        orig(self, *a, **k)
        keep["tr"] = self
    trainer.NGPTrainer.__init__ = init
    orig_step = trainer.NGPTrainer.step
    losses = []

    def step(self, *a, **k):
        r = orig_step(self, *a, **k)
        losses.append(r.sum())
        return r
    trainer.NGPTrainer.step = step
    res = MQ.product_run("cuda")
    tr = keep["tr"]
    torch.save({"params": tr.params.detach().cpu(), "density_grid": tr.density_grid.cpu(),
                "density_bitfield": tr.density_bitfield.cpu()}, os.path.join(out, "state.pt"))
    res["losses_first_300"] = [round(float(x), 6) for x in torch.stack(losses[:300]).cpu()]
    res["occupied_cells"] = int((tr.density_grid > 0).sum())
    with open(os.path.join(out, "product.json"), "w") as f:
        json.dump(res, f)
    print(json.dumps({k: res[k] for k in ("test_psnr", "test_psnr_views", "occupied_cells")}))


if __name__ == "__main__":
    main()
