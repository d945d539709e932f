#!/usr/bin/env python3
"""Run-to-run spread of the product's test PSNR on the oracle-fixture problem
(tests/golden/make_quality.py): the default and exact modes, each with the
trainer's occupancy / batch-draw seeds varied (init fixed).  One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "ar-nerf_amd")]
import make_quality as MQ  # noqa: E402


def main():
    fx = MQ.load_fixture()
    out = {"oracle": fx["test_psnr"]}
    import trainer
    orig = trainer.NGPTrainer.__init__
    for mode, kw in (("default", {}), ("exact", dict(chunk_first=0, hash_backward="atomic"))):
        res = []
        for occ_seed in (0, 1, 2):
            def init(self, *a, _s=occ_seed, **k):
                orig(self, *a, **k)
                self.occ_seed ^= 0x9E3779B97F4A7C15 * _s & 0xFFFFFFFFFFFFFFFF
            trainer.NGPTrainer.__init__ = init
            r = MQ.product_run("cuda", **kw)
            res.append(r["test_psnr"])
            print(mode, occ_seed, r["test_psnr"], r["test_psnr_views"], file=sys.stderr, flush=True)
        trainer.NGPTrainer.__init__ = orig
        out[mode] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
