#!/usr/bin/env python3
"""Standalone GPU time of the MLP kernels and the encode on a steady-state
training step's inputs (diagnostic): MLP backward full / without the weight
gradients / without the block reduction / neither (NGP_MLP_BWD_DIAG), the
colour+density MLP forward over the step's evaluated samples, and the
encode.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd"), os.path.join(ROOT, "scripts", "diag")]
import torch  # noqa: E402

import hashgrid as HG  # noqa: E402
import synthetic as S  # noqa: E402
import vren  # noqa: E402
from stages import timed  # noqa: E402
from trainer import NGPTrainer  # noqa: E402


def main():
    dev = torch.device("cuda")
    scene = S.AnalyticScene(W=800, H=800, n_images=100, scale=0.5)
    gt = scene.gt_images(device=dev)
    dirs, poses = scene.directions.to(dev), scene.poses.to(dev)
    tr = NGPTrainer(scale=0.5, batch_size=8192, device=dev)
    tr.mark_invisible_cells(scene.K, scene.poses, (scene.W, scene.H))
    for _ in range(int(os.environ.get("PRETRAIN", "1000"))):
        tr.train_step(gt, dirs, poses)
    tr.drain()
    torch.cuda.synchronize()
    p, HGL = HG._ptr, HG._lib()
    st = {"samples": int(tr.n_samples.item()), "active": int(tr.n_active_total.item())}

    def bwd():
        vren._ok(HGL.ngp_field_backward_mlp(p(tr.dirs), tr.cap, p(tr.n_active_total), p(tr.sample_idx), p(tr.enc),
                                            tr.cap, p(tr.params16), p(tr.dsig), p(tr.drgb), p(tr.denc), p(tr.grad),
                                            vren._stream()), "mlp_bwd")
    for kern in ("coop", "wave"):
        os.environ["NGP_MLP_BWD_WAVE"] = "1" if kern == "wave" else "0"
        for m, name in ((0, "full"), (1, "no_dW"), (2, "no_reduce"), (3, "no_dW_no_reduce")):
            os.environ["NGP_MLP_BWD_DIAG"] = str(m)
            st[f"mlp_bwd_{kern}_{name}" if kern != "coop" else f"mlp_bwd_{name}"] = timed(bwd)
    for k in ("NGP_MLP_BWD_DIAG", "NGP_MLP_BWD_WAVE"):
        os.environ.pop(k)
    n_all = st["samples"]
    st["mlp_fwd_all_marched"] = timed(lambda: vren._ok(HGL.ngp_field_mlp_forward(
        p(tr.enc), p(tr.dirs), tr.cap, p(tr.n_samples), None, p(tr.params16), p(tr.sigmas), p(tr.rgbs), None,
        vren._stream()), "mlp_fwd"))
    st["encode_all_marched"] = timed(lambda: vren._ok(HGL.ngp_hash_encode(
        p(tr.xyzs), tr.cap, p(tr.n_samples), None, HG.ctypes.byref(tr.grid.desc), p(tr.params16[HG.MLP_PARAMS:]),
        p(tr.enc), vren._stream()), "encode"))
    fl_f, fl_b = 20480, 59392
    st["mlp_fwd_tflops"] = round(n_all * fl_f / (st["mlp_fwd_all_marched"] * 1e-6) / 1e12, 1)
    st["mlp_bwd_tflops"] = round(st["active"] * fl_b / (st["mlp_bwd_full"] * 1e-6) / 1e12, 1)
    print(json.dumps(st))


if __name__ == "__main__":
    main()
