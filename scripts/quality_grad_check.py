#!/usr/bin/env python3
"""One training step's gradient at a TRAINED state (scripts/quality_state.py's
state.pt), product vs the reference's glue on the CPU oracle, on the same
batch (make_quality.batch(STEP)) and bitfield: the step tests compare the two
at initialisation only; this compares them where the oracle-fixture runs
diverge.
  quality_grad_check.py gpu STATE_DIR   -> STATE_DIR/grad_gpu.pt   (GPU box)
  quality_grad_check.py cpu STATE_DIR   -> STATE_DIR/grad_cpu.pt + the comparison (needs /root/reference)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "ar-nerf_amd")]
import torch  # noqa: E402

import make_quality as MQ  # noqa: E402

STEP = int(os.environ.get("STEP", "1999"))


def gpu(d):
    from trainer import NGPTrainer
    st = torch.load(os.path.join(d, "state.pt"), weights_only=True)
    dev = torch.device("cuda")
    cfg = MQ.CFG
    sc, _ = MQ.scenes()
    tr = NGPTrainer(scale=cfg["scale"], batch_size=cfg["batch"], lr=cfg["lr"], num_epochs=cfg["epochs"],
                    steps_per_epoch=cfg["steps_per_epoch"], device=dev, seed=cfg["init_seed"])
    with torch.no_grad():
        tr.params.copy_(st["params"].to(dev))
        tr.params16.copy_(tr.params.half())
        tr.density_grid.copy_(st["density_grid"].to(dev))
        tr.density_bitfield.copy_(st["density_bitfield"].to(dev))
    tr.global_step = 1  # (no occupancy update in this step)
    img, pix, noise = MQ.batch(STEP, sc)
    gt = MQ.true_div255(sc.gt_images()[img, pix])
    loss = tr.step(img.to(dev), pix.to(dev), gt.to(dev), sc.directions.to(dev), sc.poses.to(dev),
                   noise=noise.to(dev), apply_adam=False).sum()
    torch.cuda.synchronize()
    torch.save({"grad": tr.grad.cpu().clone(), "loss": float(loss), "rm": int(tr.n_samples.item())},
               os.path.join(d, "grad_gpu.pt"))
    print(json.dumps({"loss": float(loss), "rm": int(tr.n_samples.item())}))


def cpu(d):
    st = torch.load(os.path.join(d, "state.pt"), weights_only=True)
    import hashgrid as HG
    import make_golden as MG
    MG.install_stubs()
    from losses import NeRFLoss
    from models.networks import NGP
    from models.rendering import render
    vren = sys.modules["vren"]
    torch.set_num_threads(int(os.environ.get("THREADS", "8")))
    cfg = MQ.CFG
    model = NGP(cfg["scale"])
    flat = st["params"]
    nm = model.xyz_encoder.n_mlp
    with torch.no_grad():
        model.xyz_encoder.params.copy_(torch.cat([flat[:nm], flat[HG.MLP_PARAMS:]]))
        model.rgb_net.params.copy_(flat[nm:HG.MLP_PARAMS])
    model.register_buffer("density_grid", st["density_grid"].clone())
    model.density_bitfield.copy_(st["density_bitfield"])
    sc, _ = MQ.scenes()
    img, pix, noise = MQ.batch(STEP, sc)
    orig = vren.raymarching_train

    def march(*a):
        a = list(a)
        a[7] = noise
        return orig(*a)
    vren.raymarching_train = march
    o, dd = sc.rays(img, pix)
    res = render(model, o.contiguous(), dd.contiguous())
    gt = MQ.true_div255(sc.gt_images()[img, pix])
    loss_d = NeRFLoss(cfg["epochs"], "raw", cfg["scale"], 0.0, lambda_distortion=0.0)(res, {"rgb": gt})
    loss = sum(v.mean() for v in loss_d.values())
    loss.backward()
    gx, gr = model.xyz_encoder.params.grad, model.rgb_net.params.grad
    g = torch.cat([gx[:nm], gr, gx[nm:]])
    gg = torch.load(os.path.join(d, "grad_gpu.pt"), weights_only=True)
    gp = gg["grad"]
    offs = HG.HashGrid(cfg["scale"]).offsets
    groups = {"W1": (0, 2048), "W2": (2048, 3072), "rgb W3-W5": (3072, HG.MLP_PARAMS)}
    for lv in range(16):
        groups[f"L{lv}"] = (HG.MLP_PARAMS + 2 * int(offs[lv]), HG.MLP_PARAMS + 2 * int(offs[lv + 1]))
    out = {"loss_cpu": float(loss), "loss_gpu": gg["loss"], "rm_cpu": int(res["rm_samples"]), "rm_gpu": gg["rm"]}
    for k, (a, b) in groups.items():
        r, p = g[a:b].double(), gp[a:b].double()
        n = float(r.norm())
        out[k] = {"rel_l2": round(float((p - r).norm()) / max(n, 1e-30), 4),
                  "norm_ratio": round(float(p.norm()) / max(n, 1e-30), 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    {"gpu": gpu, "cpu": cpu}[sys.argv[1]](sys.argv[2])
