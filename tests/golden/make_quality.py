"""Generate tests/golden/quality_oracle.json: the REFERENCE's own training
loop glue (read from /root/reference, never copied) run on this repo's CPU
oracle in fp32 autograd -- the training-quality anchor (north_star "PSNR
within 0.2 dB of reference") that tests/test_quality_gpu.py holds the
product to.

What runs (train.py:158-200 without Lightning / apex; Lightning's
precision=16 AMP loss scaling restated, see below):
  NeRFSystem.on_train_start -> NGP.mark_invisible_cells (networks.py:209-250)
  per step: NGP.update_density_grid every 16 steps, warm-up below 256
            (networks.py:252-281, train.py:175-178);
            render(model, rays_o, rays_d) (rendering.py:13-54, train path:
            RayMarcher / VolumeRenderer autograd, white background);
            NeRFLoss 'raw' (losses.py:63-82), loss = sum of means;
            backward through the GradScaler that Trainer(precision=16)
            attaches (train.py:291 -> torch.cuda.amp.GradScaler, PyTorch's
            defaults): (loss * S).backward() with S = 2^16 initially, the
            gradients unscaled by 1/S in fp32; a step whose gradients hold
            an inf / nan is skipped (no Adam step, S halved), S doubles after
            2000 consecutive clean steps;
            FusedAdam(lr, eps=1e-15) on the model's parameters (train.py:146),
            lr = CosineAnnealingLR(num_epochs, lr/30) stepped per epoch
            (train.py:149-151)
  at the end: render(test_time=True) of held-out views (rendering.py:162-253)
            composited on white (the scene's GT background) -> mean PSNR.
with `vren` = oracle (C restatement of the .cu kernels) and `tinycudann` =
oracle.tcnn_stub (fp16 storage points, fp16 module outputs -- so the glue's
gradients into the modules, dL/dh and dL/drgb, are rounded to fp16 AT THE
LOSS SCALE S, as under AMP on the GPU -- and fp32 autograd inside the
modules) -- installed by make_golden.install_stubs.
(Rounds 1-3 ran this without the GradScaler: the fp16 boundary then flushed
gradients below 2^-24 that the reference's scaled backward keeps; those
fixtures did not model the reference and were replaced.)

Shared with the product run (tests/test_quality_gpu.py), so both train the
same problem: the scene (synthetic.AnalyticScene, TRAIN / TEST below), the
initial parameters (hashgrid.init_params, seed 4, in the reference's tcnn
layout), and every batch -- image / pixel indices and the march noise of
step k come from torch.Generator().manual_seed(BATCH_SEED + k) (the glue's
own RayMarcher noise draw is replaced by that one; distribution unchanged).
Not shared: the occupancy updates' random cells (the glue draws them from
torch's global RNG, the product from Philox on the device) -- the same
distribution; NeRF training is chaotic, so the runs are compared through
their test PSNR, not parameter by parameter.

Run:  python tests/golden/make_quality.py   (needs /root/reference; ~1 h on 8 cores)
"""
import json
import math
import os
import sys
import time

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "ar-nerf_amd")]

import torch  # noqa: E402

# the schedule (train.py's, scaled: 30 epochs x 1000 steps -> EPOCHS x STEPS_PER_EPOCH)
CFG = dict(
    scale=0.5, W=100, H=100, train_views=20, train_seed=0, test_views=4, test_seed=77,
    batch=2048, epochs=20, steps_per_epoch=100, lr=1e-2, update_interval=16, warmup_steps=256,
    init_seed=4, batch_seed=910000,
)


def scenes():
    import synthetic as S
    tr = S.AnalyticScene(W=CFG["W"], H=CFG["H"], n_images=CFG["train_views"], scale=CFG["scale"],
                         seed=CFG["train_seed"])
    te = S.AnalyticScene(W=CFG["W"], H=CFG["H"], n_images=CFG["test_views"], scale=CFG["scale"],
                         seed=CFG["test_seed"])
    return tr, te


def batch(step, sc):
    """(img, pix, noise) of training step `step` (shared with the product run)"""
    g = torch.Generator().manual_seed(CFG["batch_seed"] + step)
    img, pix = sc.sample_batch(CFG["batch"], g)
    noise = torch.rand(CFG["batch"], generator=g)
    return img, pix, noise


def lr_at(step):
    e = step // CFG["steps_per_epoch"]
    lo = CFG["lr"] / 30
    return lo + (CFG["lr"] - lo) * (1 + math.cos(math.pi * e / CFG["epochs"])) / 2


def true_div255(u8):
    x = u8.float()
    return x / torch.full_like(x, 255.0)


def test_psnr(render_fn, te):
    """mean PSNR of the held-out views; render_fn(o, d) -> (rgb composited on
    black, opacity); the white background is added here"""
    gt = true_div255(te.gt_images())
    ps = []
    for i in range(te.poses.shape[0]):
        P = te.poses[i]
        d = (te.directions @ P[:, :3].t()).contiguous()
        o = P[:, 3].expand_as(d).contiguous()
        rgb, op = render_fn(o, d)
        rgb = (rgb.cpu() + (1 - op.cpu())[:, None]).clamp(0, 1)
        mse = float(torch.mean((rgb - gt[i]) ** 2))
        ps.append(-10 * math.log10(max(mse, 1e-12)))
    return sum(ps) / len(ps), ps


def product_run(device="cuda", steps=None, **trainer_kw):
    """The product (trainer.NGPTrainer on the device) on the same problem:
    same scene, init (NGPTrainer seed 4 = hashgrid.init_params seed 4), lr
    schedule and batches (img, pix, noise of each step given to step());
    occupancy updates by the trainer itself.  Test PSNR through
    NGPTrainer.render (rendering.py:162-253's loop on the native kernels),
    composited on white as above.  trainer_kw: e.g. the exact mode
    (chunk_first=0, hash_backward='atomic').  -> dict"""
    from trainer import NGPTrainer
    dev = torch.device(device)
    sc, te = scenes()
    n_steps = steps if steps is not None else CFG["epochs"] * CFG["steps_per_epoch"]
    tr = NGPTrainer(scale=CFG["scale"], batch_size=CFG["batch"], lr=CFG["lr"], num_epochs=CFG["epochs"],
                    steps_per_epoch=CFG["steps_per_epoch"], update_interval=CFG["update_interval"],
                    warmup_steps=CFG["warmup_steps"], seed=CFG["init_seed"], device=dev, **trainer_kw)
    tr.mark_invisible_cells(sc.K, sc.poses, (sc.W, sc.H))
    gt_u8 = sc.gt_images(device=dev)
    dirs, poses = sc.directions.to(dev), sc.poses.to(dev)
    losses = []
    t0 = time.time()
    for step in range(n_steps):
        img, pix, noise = batch(step, sc)
        img_d, pix_d = img.to(dev), pix.to(dev)
        rgb_gt = true_div255(gt_u8[img_d, pix_d])
        losses.append(tr.step(img_d, pix_d, rgb_gt, dirs, poses, noise=noise.to(dev)).sum())
    torch.cuda.synchronize()
    wall = time.time() - t0
    psnr, per_view = test_psnr(lambda o, d: (lambda r: (r["rgb"], r["opacity"]))(tr.render(o.to(dev), d.to(dev))),
                               te)
    ls = torch.stack(losses).cpu()
    return {"test_psnr": round(psnr, 4), "test_psnr_views": [round(x, 4) for x in per_view],
            "final_loss_mean_last_100": float(ls[-100:].mean()), "loss_curve_every_50": ls[::50].tolist(),
            "train_wall_s": round(wall, 2), "steps": n_steps}


def load_fixture():
    with open(os.path.join(HERE, "quality_oracle.json")) as f:
        return json.load(f)


def _patch_f32_outputs(O):
    """tinycudann's torch modules return fp16 (tcnn's output precision), so in
    the reference the gradients the glue hands back to them -- dL/dh from
    TruncExp (custom_functions.py:162-173, computed in fp32 under autocast and
    cast back across the fp16 output) and dL/drgb from VolumeRenderer -- are
    rounded to fp16 (at the GradScaler's loss scale under Lightning's
    precision=16, train.py:291: the reference-precision fixtures model that
    scaler, see the GradScaler model further down).  This variant -- the "fp32 boundary" fixture --
    returns the same VALUES (fp16-rounded) as fp32 tensors, so those
    gradients stay fp32 and no rounding happens at the boundary at all.  On the CPU (no autocast) TruncExp then also
    runs in fp32, as it does on the GPU."""
    T = O.tcnn_stub

    def nwe_forward(self, x01):
        Ws, _ = O.mlp_layers(self.params[:self.n_mlp], self.dims)
        enc = O._HashEncodeFn.apply(self.params[self.n_mlp:], x01.float().contiguous(), self.spec, self._mn, self._mx)
        return O.mlp_forward(enc, Ws)

    def net_forward(self, x):
        Ws, _ = O.mlp_layers(self.params, self.dims)
        out = O.mlp_forward(x.float(), Ws)[:, :self.n_out]
        if self.act == "Sigmoid":
            out = O.rh(torch.sigmoid(out))
        return out
    T.NetworkWithInputEncoding.forward = nwe_forward
    T.Network.forward = net_forward


def main():
    import hashgrid as HG  # (the product's init: before the stubs replace `vren`)
    flat = HG.init_params(HG.HashGrid(CFG["scale"]), seed=CFG["init_seed"], device="cpu")
    import make_golden as MG
    MG.install_stubs()
    import oracle as O
    f32_out = os.environ.get("TCNN_OUT", "f16") == "f32"
    if f32_out:  # (variant) the tcnn modules hand fp32 outputs to the glue: no fp16 rounding of dL/dh, dL/drgb
        _patch_f32_outputs(O)
    vren = sys.modules["vren"]
    from losses import NeRFLoss
    from models.networks import NGP
    from models.rendering import render
    torch.set_num_threads(int(os.environ.get("THREADS", min(8, os.cpu_count() or 1))))
    nthreads = torch.get_num_threads()
    sc, te = scenes()
    model = NGP(CFG["scale"])
    G = model.grid_size
    ax = torch.arange(G, dtype=torch.int32)
    model.register_buffer("density_grid", torch.zeros(model.cascades, G ** 3))
    model.register_buffer("grid_coords", torch.stack(torch.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3))
    # the product's initial parameters in the tcnn layout
    nm = model.xyz_encoder.n_mlp
    with torch.no_grad():
        model.xyz_encoder.params.copy_(torch.cat([flat[:nm], flat[HG.MLP_PARAMS:]]))
        model.rgb_net.params.copy_(flat[nm:HG.MLP_PARAMS])
    params = [p for p in model.parameters() if p is not None and p.requires_grad]
    state = {p: (torch.zeros_like(p), torch.zeros_like(p)) for p in params}
    model.mark_invisible_cells(sc.K, sc.poses, (sc.W, sc.H))
    gt_u8 = sc.gt_images()
    loss_fn = NeRFLoss(CFG["epochs"], "raw", CFG["scale"], 0.0, lambda_distortion=0.0)
    cur_noise = {}
    orig_march = vren.raymarching_train

    def march(*a):  # RayMarcher's noise -> the shared batch noise of this step
        a = list(a)
        a[7] = cur_noise["n"]
        return orig_march(*a)
    vren.raymarching_train = march
    thr = 0.01 * 1024 / 3 ** 0.5
    n_steps = CFG["epochs"] * CFG["steps_per_epoch"]
    losses, t0 = [], time.time()
    # Lightning precision=16 (train.py:291): torch.cuda.amp.GradScaler with its defaults
    # (init_scale 2^16, growth 2 every 2000 clean steps, backoff 0.5).  The fp32-boundary
    # variant needs no scale (a power-of-two scale is exact there).
    use_scaler = os.environ.get("GRAD_SCALER", "1") == "1" and not f32_out
    scaler = dict(scale=65536.0 if use_scaler else 1.0, growth_tracker=0, skipped=[], adam_steps=0)
    occ = int(os.environ.get("OCC_SEED", "0"))  # (spread runs: other occupancy draws)
    torch.manual_seed(CFG["batch_seed"] - 1 - occ)  # the glue's occupancy draws
    for step in range(n_steps):
        if step % CFG["update_interval"] == 0:
            # index_put_ with duplicate cells races on several CPU threads (make_golden.main)
            torch.set_num_threads(1)
            model.update_density_grid(thr, warmup=step < CFG["warmup_steps"])
            torch.set_num_threads(nthreads)
        img, pix, noise = batch(step, sc)
        o, d = sc.rays(img, pix)
        cur_noise["n"] = noise
        res = render(model, o.contiguous(), d.contiguous())
        gt = true_div255(gt_u8[img, pix])
        loss_d = loss_fn(res, {"rgb": gt})
        loss = sum(v.mean() for v in loss_d.values())
        for p in params:
            p.grad = None
        S = scaler["scale"]
        (loss * S if use_scaler else loss).backward()
        lr = lr_at(step)
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in params]
        # GradScaler.unscale_: grads * (1/S) in fp32, found_inf over all of them
        found_inf = use_scaler and not all(bool(torch.isfinite(g).all()) for g in grads)
        if found_inf:  # GradScaler.step skips optimizer.step(); update() halves the scale
            scaler["skipped"].append(step)
            scaler["scale"] = S * 0.5
            scaler["growth_tracker"] = 0
        else:
            inv = 1.0 / S
            scaler["adam_steps"] += 1
            for p, g in zip(params, grads):
                m, v = state[p]
                O.adam_(p.data, (g * inv if use_scaler else g).contiguous(), m, v, lr, scaler["adam_steps"])
            if use_scaler:
                scaler["growth_tracker"] += 1
                if scaler["growth_tracker"] == 2000:
                    scaler["scale"] = S * 2.0
                    scaler["growth_tracker"] = 0
        losses.append(float(loss.detach()))
        if step % 50 == 0 or step == n_steps - 1:
            print(f"[make_quality] step {step} loss {losses[-1]:.5f} rm_s {int(res['rm_samples']) / CFG['batch']:.1f} "
                  f"elapsed {time.time() - t0:.0f}s", flush=True)
    vren.raymarching_train = orig_march

    def rf(o, d):
        with torch.no_grad():
            r = render(model, o, d, test_time=True, blend_bkg=False)
        return r["rgb"], r["opacity"]
    psnr, per_view = test_psnr(rf, te)
    out = {"cfg": CFG, "test_psnr": round(psnr, 4), "test_psnr_views": [round(x, 4) for x in per_view],
           "loss_curve_every_50": [round(x, 6) for x in losses[::50]],
           "final_loss_mean_last_100": sum(losses[-100:]) / 100,
           "occupied_cells": int((model.density_grid > 0).sum()),
           "cpu_threads": nthreads, "wall_s": round(time.time() - t0, 1), "occ_seed": occ,
           "what": "reference train.py loop glue + oracle fp32-autograd kernels (make_quality.py)"}
    out["tcnn_out"] = "f32" if f32_out else "f16"
    out["grad_scaler"] = ({"init_scale": 65536.0, "final_scale": scaler["scale"], "skipped_steps": scaler["skipped"],
                           "adam_steps": scaler["adam_steps"], "growth_interval": 2000, "backoff": 0.5,
                           "what": "Lightning precision=16 (train.py:291): torch.cuda.amp.GradScaler defaults"}
                          if use_scaler else None)
    name = "quality_oracle" + ("" if occ == 0 else f"_occ{occ}") + ("_f32out" if f32_out else "")
    path = os.path.join(HERE, name + ".json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("test_psnr", "test_psnr_views", "wall_s")}))


if __name__ == "__main__":
    main()
