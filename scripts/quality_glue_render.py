#!/usr/bin/env python3
"""Render a trained state saved by scripts/quality_state.py (the product's
parameters, density grid and bitfield after the oracle-fixture schedule)
through the reference's own test-time glue (models/rendering.py:162-253 with
the CPU oracle as vren / tinycudann, make_golden.install_stubs) and print the
held-out PSNR next to the product's own render of the same state.  Needs
/root/reference (this container only).
usage: quality_glue_render.py STATE_DIR"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "ar-nerf_amd")]
import torch  # noqa: E402

import make_quality as MQ  # noqa: E402


def main():
    d = sys.argv[1]
    st = torch.load(os.path.join(d, "state.pt"), weights_only=True)
    prod = json.load(open(os.path.join(d, "product.json")))
    import hashgrid as HG
    import make_golden as MG
    MG.install_stubs()
    from models.networks import NGP
    from models.rendering import render
    torch.set_num_threads(int(os.environ.get("THREADS", "8")))
    cfg = MQ.CFG
    model = NGP(cfg["scale"])
    G = model.grid_size
    flat = st["params"]
    nm = model.xyz_encoder.n_mlp
    with torch.no_grad():
        model.xyz_encoder.params.copy_(torch.cat([flat[:nm], flat[HG.MLP_PARAMS:]]))
        model.rgb_net.params.copy_(flat[nm:HG.MLP_PARAMS])
    model.register_buffer("density_grid", st["density_grid"].clone())
    model.density_bitfield.copy_(st["density_bitfield"])
    _, te = MQ.scenes()

    def rf(o, dd):
        with torch.no_grad():
            r = render(model, o, dd, test_time=True, blend_bkg=False)
        return r["rgb"], r["opacity"]
    psnr, views = MQ.test_psnr(rf, te)
    out = {"glue_render_of_product_state": round(psnr, 4), "views": [round(v, 4) for v in views],
           "product_render": prod["test_psnr"], "product_views": prod["test_psnr_views"],
           "oracle_fixture": MQ.load_fixture()["test_psnr"]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
