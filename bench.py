#!/usr/bin/env python3
"""Training-throughput benchmark of the MI355X-native Instant-NGP hot path.

Metric (BASELINE.json): training rays/s on Lego-shaped 8192-ray batches
(L=16, T=2^19 hash, 64-wide MLPs, 128^3 occupancy grid, fp16 field), one
process per GPU, each rank drawing its own 8192-ray batch (the reference's
Lightning DDP semantics, train.py:288) -> weak scaling, value = all ranks'
rays / max-over-ranks wall time.

Workload: no dataset is reachable, so the scene is analytic
(synthetic.AnalyticScene: 100 800x800 views of an opaque sphere + box on
white, Lego camera intrinsics); the model is first trained for --pretrain
steps (setup, untimed) so the occupancy grid and samples/ray are in the
steady state of real training, then --warmup untimed and --steps timed FULL
training steps (occupancy update every 16 steps, ray generation, marching,
field fwd/bwd, compositing + loss, [RCCL all-reduce], Adam).

Run: python bench.py [--gpus N --steps K --warmup W]; for N>1 under
torch.distributed.run (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* from the env).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import ktimer as KT  # noqa: E402
import vren  # noqa: E402
import synthetic as S  # noqa: E402
from trainer import NGPTrainer  # noqa: E402

with open(os.path.join(ROOT, "BASELINE.json")) as f:
    BASELINE = json.load(f)

# Algorithmic work per unit, per op of the step (DESIGN.md
# §6-7).  Units: "marched" / "evaluated" (field-evaluated) / "composited" /
# "active" (gradient-carrying) samples of the step, "params" of the model.
# bound: "hbm" (algorithmic bytes vs 8 TB/s), "mfma" (dense fp16 FLOPs vs
# 2.5 PFLOP/s), "atomic" (bytes added by memory-side float atomics vs the
# chip-wide ~1.3 TB/s of MI355X_MICROARCH.md "Global float atomics").
# Members are device-probe names (ktimer.PROBES): an op's time is the sum of
# its kernels' execution spans, as a rocprofv3 kernel trace measures them.
#  hash_encode (both forward rounds): 16 levels x 8 corners x 2 feats x 2 B
#      gathered (512 B) + xyz 12 B + fp16 features 64 B (§8(d))   -> 588 B
#      (+ the fused MLP forward, density 32-64-16 + colour 32-64-64-16:
#      20,480 FLOP, noted beside it)
#  mlp_bwd: forward recompute + dX + dW of both MLPs               -> 59,392 FLOP
#  hash_bwd_coarse (levels 0-7, memory-side atomics): 8 levels x 8 corners
#      x 2 fp32 gradients added                                    -> 512 B
#  hash_bwd_fine = hash_write + hash_accum (levels 8-15, §8(d)'s hash
#      backward restricted to them): dL/dfeat 32 B + xyz 12 B + read-modify-
#      write of 8 x 8 x 2 fp16-sized table gradients (2 x 256 B)  -> 556 B,
#      plus, with the binned levels' Adam fused into the accumulation, their
#      Adam state: p, m, v read and written + the fp16 shadow     -> 26 B / param
#      (the counting sort's records are implementation traffic: roofline.traffic)
#  march: xyz, dir, t, dt written (32 B / marched sample)
#  composite_loss: fwd 28 B + bwd 48 B per composited sample      -> 76 B
#  adam: p, g, m, v read; p, m, v, fp16 p written, g zeroed        -> 34 B / param
_MLP_FWD = 2 * (32 * 64 + 64 * 16) + 2 * (32 * 64 + 64 * 64 + 64 * 16)
_MLP_BWD = (2 * (32 * 64 + 64 * 16 + 32 * 64 + 64 * 64 + 64 * 16)
            + 2 * (16 * 64 + 64 * 64 + 64 * 16 + 16 * 64 + 64 * 32)
            + 2 * (16 * 64 + 64 * 64 + 64 * 32 + 16 * 64 + 64 * 32))
KERNEL_WORK = {  # name: (bound, [(work per unit, unit basis), ...], member probes)
    "hash_encode": ("hbm", [(16 * 8 * 2 * 2 + 12 + 64, "evaluated")], ["first_chunk", "field_encode_mlp", "pre_encode"]),
    "mlp_bwd": ("mfma", [(_MLP_BWD, "active")], ["mlp_bwd"]),
    # the fused MLP forward's MFMA fraction over its launches' whole span (the same launches as
    # hash_encode's rounds: the gathers share the time, so this is a lower bound on the MLP's own)
    "mlp_fwd": ("mfma", [(_MLP_FWD, "evaluated")], ["first_chunk", "field_encode_mlp"]),
    "hash_bwd_coarse": ("atomic", [(8 * 8 * 2 * 4, "active")], ["hash_bwd_coarse"]),
    "hash_bwd_fine": ("hbm", [(32 + 12 + 2 * 8 * 8 * 2 * 2, "active"), (26, "fused_params")],
                      ["hash_write", "hash_accum"]),
    "march": ("hbm", [(32, "marched")], ["march"]),
    "composite_loss": ("hbm", [(76, "composited")], ["composite_loss"]),
    "adam": ("hbm", [(34, "adam_params")], ["adam"]),  # params the Adam launches step
}
# PMC traffic (profiles/pmc_traffic.json) keys of each op's kernels
PMC_KEYS = {"hash_bwd_fine": ["hash_write", "hash_accum"], "hash_encode": ["hash_encode_first", "hash_encode", "hash_encode_pre"],
            "mlp_bwd": ["mlp_bwd"], "adam": ["adam"]}


PEAK = {"hbm": (8000.0, "GB/s"), "mfma": (2500.0, "TFLOP/s"), "atomic": (1300.0, "GB/s")}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=800)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--pretrain", type=int, default=2000, help="untimed setup training steps (steady-state occupancy)")
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--scale", type=float, default=0.5)
    ap.add_argument("--res", type=int, default=800)
    ap.add_argument("--images", type=int, default=100)
    ap.add_argument("--psnr-views", type=int, default=2)
    ap.add_argument("--psnr-res", type=int, default=400)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--breakdown-steps", type=int, default=100,
                    help="graph-replayed steps with HIP events around every kernel (per-kernel breakdown)")
    ap.add_argument("--hash-backward", default="hybrid", choices=["hybrid", "binned", "atomic"])
    ap.add_argument("--bin-level-lo", type=int, default=None,
                    help="hybrid hash backward: first binned level (default: trainer's, 8 / 0 for cascaded scenes)")
    ap.add_argument("--emulate-dp", type=int, default=0, metavar="N",
                    help="(world 1) run the data-parallel step of a world of N ranks as rank 0 -- graph segments, "
                         "ZeRO-1 shards of 1/N, per-bucket reduce-scatter / sharded Adam / all-gather on the comm "
                         "stream -- with the collectives as local copies: one rank's compute at world N without "
                         "the xGMI transfers (only shard 0 is stepped: a timing mode)")
    ap.add_argument("--dp-fine-buckets", type=int, default=None,
                    help="world > 1 (or --emulate-dp): ZeRO-1 buckets of the binned hash levels (default: trainer's)")
    ap.add_argument("--chunk-first", type=int, default=None,
                    help="chunked field evaluation: first round's samples per row (0: every marched sample in one "
                         "launch; default: trainer's, 64)")
    ap.add_argument("--no-pair-steps", action="store_true",
                    help="one steady-state step per graph replay (default: two consecutive steps per replay, "
                         "trainer pair_steps: one replay boundary per two steps, +1.1 %, 5 of 5 pairs, "
                         "profiles/r03/ab/pair_steps_r3d.txt)")
    ap.add_argument("--bin-merge-hi", type=int, default=None,
                    help="binned levels below this merge runs of equal corner pairs along a ray (default: "
                         "trainer's, 11 / 16 for cascaded scenes)")
    ap.add_argument("--bin-samples-per-ray", type=int, default=None,
                    help="binned hash-backward workspace per ray (default: trainer's, 128 / 512 for cascaded scenes)")
    ap.add_argument("--erode", default="auto", choices=["auto", "on", "off"],
                    help="occupancy erode decay (networks.py:270-272); auto = on for cascaded (garden-shaped, "
                         "COLMAP-like) scenes as train.py:178 does for colmap")
    ap.add_argument("--quality-steps", type=int, default=30000,
                    help="test-PSNR check after the reference schedule (scripts/quality_30k.py: product defaults vs "
                         "exact mode, each in a child process; 0: skip)")
    ap.add_argument("--no-oracle-quality", action="store_true",
                    help="skip the test-PSNR check against the fp32-oracle fixtures (tests/golden/make_quality.py: "
                         "2000 steps of the reference's schedule on a small problem, product defaults and exact mode)")
    ap.add_argument("--infer-frames", type=int, default=20, help="timed full-frame test renders (0: skip)")
    ap.add_argument("--infer-res", type=int, default=800)
    ap.add_argument("--dropin-steps", type=int, default=50,
                    help="timed steps of the reference's loop on the drop-in surface (DropinLoop; 0: skip)")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="world > 1 process group (nccl = RCCL; gloo only to rehearse the path with ranks sharing a GPU)")
    return ap.parse_args()


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # (--dist-backend gloo with more ranks than GPUs: a rehearsal of the world > 1 bench
        # path on a one-GPU box, ranks sharing the card; the measured path is RCCL, one GPU per rank)
        dev = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(args.dist_backend)
    else:
        torch.cuda.set_device(0)
    return world, rank, torch.cuda.current_device()


def psnr_eval(trainer, scene, n_views, res, seed=123):
    """Test PSNR on held-out analytic views (black test background like
    models/rendering.py:240 would need a black GT; the analytic GT is on
    white, so the white background is blended: bg=1)."""
    sc = S.AnalyticScene(W=res, H=res, n_images=n_views, scale=scene.scale, seed=seed)
    psnrs = []
    for i in range(n_views):
        P = sc.poses[i].cuda()
        d = (sc.directions.cuda() @ P[:, :3].t()).contiguous()
        o = P[:, 3].expand_as(d).contiguous()
        out = trainer.render(o, d, bg=1.0)
        gt = sc.gt_rgb_rays(o, d)
        mse = torch.mean((out["rgb"].clamp(0, 1) - gt) ** 2).item()
        psnrs.append(-10 * math.log10(max(mse, 1e-12)))
    return sum(psnrs) / len(psnrs)


def inference_bench(trainer, res, frames, world, rank, iters_per_graph=24, iters_tail=4):
    """BASELINE config 5: full-frame test-time render (models/rendering.py:162-253)
    of the trained model, graph-captured (renderer.TestRenderer), `frames` poses
    per rank (frames are independent: replicas).  The host-driven loop
    (trainer.render, the reference's control flow) is timed on one frame beside it."""
    import renderer as RD
    sc = S.AnalyticScene(W=res, H=res, n_images=max(2, frames), scale=trainer.scale, seed=321 + rank)
    n = res * res
    rr = RD.TestRenderer(n, trainer.grid, trainer.params16, trainer.density_bitfield, trainer.cascades,
                         trainer.scale, trainer.G, exp_step_factor=trainer.esf, iters_per_graph=iters_per_graph,
                         iters_tail=iters_tail)
    rr.set_camera(sc.directions.cuda(), trainer.center, trainer.half_size)
    poses = sc.poses.cuda()
    for i in range(2):  # capture + warm
        rr.render_pose(poses[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    iters = samples = 0
    for i in range(frames):
        out = rr.render_pose(poses[i % poses.shape[0]])
        iters += rr.last_iterations
        samples += int(out["total_samples"])
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([t], device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
    # the host-driven loop on the last pose, same rays
    o, d = rr.rays_o.clone(), rr.rays_d.clone()
    trainer.render(o, d)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ref = trainer.render(o, d)
    torch.cuda.synchronize()
    t_host = time.perf_counter() - t1
    same = bool(torch.equal(ref["rgb"], out["rgb"]) and torch.equal(ref["opacity"], out["opacity"]))
    return {"fps": round(world * frames / t, 2), "ms_per_frame": round(t / frames * 1e3, 3), "frames_per_rank": frames,
            "resolution": [res, res], "n_gpus": world, "iterations_per_frame": round(iters / frames, 1),
            "samples_per_ray": round(samples / (frames * n), 2), "graphs": True,
            # the trained state (hence samples/ray) varies run to run: these two are the comparable figures
            "ms_per_frame_per_sample_per_ray": round(t / frames * 1e3 / max(samples / (frames * n), 1e-9), 4),
            "samples_per_s": round(world * samples / t),
            "host_loop_ms_per_frame": round(t_host * 1e3, 3), "host_loop_bit_exact": same,
            "workload": "full-frame test render of the trained model (black bg), march+field+composite per "
                        f"iteration in HIP graphs ({iters_per_graph} iterations, then {iters_tail} per replay while rays "
                        "remain), one host sync per graph"}


class DropinLoop:
    """The reference's training loop on the drop-in surface, as a user who
    swaps the package in behind train.py gets it: NeRFSystem.forward
    (train.py:84-108: poses / directions gathered per ray, get_rays,
    models.rendering.render_rays) + training_step (train.py:158-200:
    update_density_grid every 16 steps, NeRFLoss, loss = sum of means) +
    Lightning's backward + FusedAdam (train.py:146-152, optimizers.FusedAdam)
    on models.networks.NGP.  Batches are drawn as the reference's dataset
    draws them (a random image and pixel per ray, datasets/base.py:22-35) but
    with the indices drawn on the device and the images resident in HBM.
    Starts from `trainer`'s state (parameters, occupancy grid, Adam moments
    and step)."""

    def __init__(self, trainer, gt_images, directions, poses, batch, seed=7):
        from datasets.ray_utils import get_rays
        from losses import NeRFLoss
        from models.networks import NGP
        from models.rendering import render_rays
        from optimizers import FusedAdam
        dev = trainer.dev
        self.get_rays, self.render_rays = get_rays, render_rays
        m = NGP(trainer.scale).to(dev)
        with torch.no_grad():
            m.params.copy_(trainer.params)
        m.density_bitfield.copy_(trainer.density_bitfield)
        m.register_buffer("density_grid", trainer.density_grid.clone())  # train.py:78-80
        m.register_buffer("grid_coords", trainer.grid_coords.clone())
        self.model = m
        self.opt = FusedAdam([m.params], trainer.lr(), eps=1e-15)
        st = self.opt.state[m.params]
        st["step"] = int(trainer.dctr[0].item())
        st["exp_avg"], st["exp_avg_sq"] = trainer.exp_avg.clone(), trainer.exp_avg_sq.clone()
        self.loss = NeRFLoss(30, "raw", trainer.scale, 0.0, lambda_distortion=0.0)
        self.gt, self.directions, self.poses, self.batch = gt_images, directions, poses, batch
        self.global_step = trainer.global_step
        self.gen = torch.Generator(device=dev).manual_seed(seed)
        self.kw = {"exp_step_factor": 1 / 256} if trainer.scale > 0.5 else {}

    def step(self):
        m, B = self.model, self.batch
        if self.global_step % 16 == 0:
            m.update_density_grid(0.01 * 1024 / 3 ** 0.5, warmup=False)
        img = torch.randint(self.gt.shape[0], (B,), device=self.gt.device, generator=self.gen)
        pix = torch.randint(self.gt.shape[1], (B,), device=self.gt.device, generator=self.gen)
        rays_o, rays_d = self.get_rays(self.directions[pix], self.poses[img])
        results = self.render_rays(m, rays_o, rays_d, test_time=False, random_bg=False, **self.kw)
        rgb = self.gt[img, pix].float() / 255
        loss_d = self.loss(results, {"rgb": rgb}, step=self.global_step)
        loss = sum(lo.mean() for lo in loss_d.values())
        loss.backward()
        self.opt.step()
        self.opt.zero_grad()  # (torch's default, set_to_none=True: the next backward assigns the gradient)
        self.global_step += 1
        return loss, results


def dropin_bench(trainer, gt_images, directions, poses, batch, steps, warmup=5):
    """rays/s of DropinLoop (the reference's loop on the drop-in surface),
    `steps` timed after `warmup`; same trained state as the product line."""
    loop = DropinLoop(trainer, gt_images, directions, poses, batch)
    for _ in range(warmup):
        loop.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rm = vr = 0
    for _ in range(steps):
        loss, res = loop.step()
        rm += res["rm_samples"]
        vr += res["vr_samples"]
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    return {"value": round(batch * steps / t, 1), "unit": "rays/s", "steps": steps, "warmup": warmup,
            "ms_per_step": round(t / steps * 1e3, 3), "rm_samples_per_ray": round(float(rm) / (steps * batch), 2),
            "vr_samples_per_ray": round(float(vr) / (steps * batch), 2), "last_loss": round(float(loss), 5),
            "loop": "models.rendering.render_rays + losses.NeRFLoss + loss.backward() + optimizers.FusedAdam on "
                    "models.networks.NGP, update_density_grid every 16 steps (train.py:84-200), eager, from the "
                    "product run's trained state"}


def oracle_quality():
    """J1 (north_star "PSNR within 0.2 dB of reference"): the product trained
    on the fp32-oracle fixture problem (tests/golden/make_quality.py: the
    reference's training-loop glue on the CPU oracle, 2000 steps of 2048 rays,
    same scene / init / batches), defaults and exact mode, against the
    committed fixtures: the oracle at the reference's precision (fp16
    tcnn-module boundary under Lightning precision=16's GradScaler,
    train.py:291; three occupancy draws) and with that boundary in fp32.
    Fixtures are data (JSON); the oracle itself does not run here."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_quality as MQ

    def fx(name):
        p = os.path.join(ROOT, "tests", "golden", name)
        return json.load(open(p))["test_psnr"] if os.path.exists(p) else None
    ref = [v for v in (fx("quality_oracle.json"), fx("quality_oracle_occ1.json"), fx("quality_oracle_occ2.json"))
           if v is not None]
    f32 = fx("quality_oracle_f32out.json")
    out = {"oracle_fp32_boundary": f32, "oracle_reference_precision": ref, "steps": MQ.CFG["epochs"] *
           MQ.CFG["steps_per_epoch"], "problem": "analytic scene 100x100, 20 train / 4 test views, 2048-ray batches"}
    for mode, kw in (("default", {}), ("exact", dict(chunk_first=0, hash_backward="atomic"))):
        r = MQ.product_run("cuda", **kw)
        out[f"product_{mode}"] = r["test_psnr"]
        if f32 is not None:
            out[f"delta_{mode}_vs_fp32_boundary_db"] = round(r["test_psnr"] - f32, 3)
        if ref:
            out[f"delta_{mode}_vs_reference_precision_mean_db"] = round(r["test_psnr"] - sum(ref) / len(ref), 3)
            out[f"{mode}_within_0.2_db_of_reference_precision"] = bool(min(ref) - 0.2 <= r["test_psnr"] <= max(ref) + 0.2)
    return out


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(trainer, scene, gt_images, batch, warm=3, timed=20):
    """The oracle (oracle/, the CPU restatement of the reference's kernels +
    torch fp32 autograd MLPs) timed on this host on the same workload: full
    training steps on `batch`-ray batches from the trained model state,
    `warm` untimed then `timed` timed, median step time.
    Threads: the host cores this process may use (OMP_NUM_THREADS when set --
    the GPU box's share -- else all cores)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # test/baseline infrastructure only
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(threads)
    ot = O.OracleTrainer(trainer.params, scene.scale, trainer.density_bitfield, trainer.cascades)
    gen = torch.Generator().manual_seed(77)
    c = torch.zeros(1, 3); h = torch.ones(1, 3) * scene.scale
    times, samples = [], 0
    for i in range(warm + timed):
        img, pix = scene.sample_batch(batch, gen)
        o, d = scene.rays(img, pix)
        _, ht, _ = O.ray_aabb_intersect(o, d, c, h, 1)
        ht = ht[:, 0].contiguous()
        ht[(ht[:, 0] >= 0) & (ht[:, 0] < 0.01), 0] = 0.01
        gt = gt_images[img.to(gt_images.device), pix.to(gt_images.device)].float().cpu() / 255
        noise = torch.rand(batch, generator=gen)
        t0 = time.perf_counter()
        _, n = ot.step(o.contiguous(), d.contiguous(), ht, gt, noise, torch.ones(3))
        if i >= warm:
            times.append(time.perf_counter() - t0)
            samples += n
    times.sort()
    med = times[len(times) // 2] if len(times) % 2 else 0.5 * (times[len(times) // 2 - 1] + times[len(times) // 2])
    return {"value": round(batch / med, 1), "unit": "rays/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"median of {timed} full training steps of the {batch}-ray batch after {warm} warm-up steps "
                      f"on the oracle (C march/composite/hash + torch fp32 MLP autograd + C Adam over all "
                      f"{trainer.params.numel()} params), {samples / max(1, timed) / batch:.1f} samples/ray, "
                      f"{sum(times):.1f} s timed"}


def pmc_traffic(members):
    """HBM bytes per step of the op made of kernels `members` (PMC keys, one
    launch per step each), from the committed PMC summary
    (profiles/pmc_traffic.json, written by scripts/pmc_traffic.py from
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this bench,
    corrected per MI355X_MICROARCH.md "HBM"), or None if not measured."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    if not members or not all(m in t for m in members):
        return None
    return round(sum(t[m]["bytes_per_launch"] for m in members))


def transplant_state(src, dst):
    """Training state of trainer src into dst (same scene and model shape): parameters, fp16 shadow,
    Adam moments, occupancy grid / bitfield / threshold, device counters and the host step count."""
    n = src.params.numel()
    with torch.no_grad():
        dst.params[:n].copy_(src.params)
        dst.params16[:n].copy_(src.params16)
        dst.exp_avg[:n].copy_(src.exp_avg[:n])
        dst.exp_avg_sq[:n].copy_(src.exp_avg_sq[:n])
        for name in ("density_grid", "density_bitfield", "threshold", "dctr"):
            getattr(dst, name).copy_(getattr(src, name))
    dst.global_step = src.global_step
    dst._updated_for = src._updated_for
    dst.invalidate_pre_encode()


def main():
    args = parse()
    world, rank, local = setup_dist(args)  # local: this rank's device index
    dev = torch.device("cuda", local)
    torch.manual_seed(0)
    scene = S.AnalyticScene(W=args.res, H=args.res, n_images=args.images, scale=args.scale)
    gt_images = scene.gt_images(device=dev)  # (n_img, HW, 3) u8, resident in HBM
    directions = scene.directions.to(dev).contiguous()
    poses = scene.poses.to(dev).contiguous()
    erode = args.erode == "on" or (args.erode == "auto" and args.scale > 0.5)
    trainer = NGPTrainer(scale=args.scale, batch_size=args.batch, device=dev, hash_backward=args.hash_backward,
                         bin_level_lo=args.bin_level_lo, bin_samples_per_ray=args.bin_samples_per_ray, erode=erode,
                         bin_merge_hi=args.bin_merge_hi, pair_steps=not args.no_pair_steps, emulate_dp=args.emulate_dp,
                         **({} if args.dp_fine_buckets is None else {"dp_fine_buckets": args.dp_fine_buckets}),
                         **({} if args.chunk_first is None else {"chunk_first": args.chunk_first}))
    trainer.mark_invisible_cells(scene.K, scene.poses, (scene.W, scene.H))
    WORK = KERNEL_WORK
    R = args.batch

    def run(n):
        """Exactly n training steps, each on a batch drawn on device
        (trainer.train_step: pixels, ground truth and noise from a counter-based
        RNG); batch i+1 is drawn and marched on the side stream during step i.
        The last call never starts a two-step replay, so no step of this window
        runs in the next one (nor one of the previous window in this one)."""
        for i in range(n):
            trainer.train_step(gt_images, directions, poses, allow_pair=i < n - 1)
        trainer.drain()

    def adam_steps():
        """steps completed on the device so far (the device step counter; call
        after a synchronize)"""
        return int(trainer.dctr[0].item())

    t0 = time.time()
    if args.emulate_dp:
        # One emulated rank updates only its shards (the other ranks' updates never arrive), so it
        # would train a different model with different work per step: the setup steps run on a
        # single-process trainer and its whole state moves into the emulated rank before timing.
        pre = NGPTrainer(scale=args.scale, batch_size=args.batch, device=dev, hash_backward=args.hash_backward,
                         bin_level_lo=args.bin_level_lo, bin_samples_per_ray=args.bin_samples_per_ray, erode=erode,
                         bin_merge_hi=args.bin_merge_hi, pair_steps=not args.no_pair_steps,
                         **({} if args.chunk_first is None else {"chunk_first": args.chunk_first}))
        pre.mark_invisible_cells(scene.K, scene.poses, (scene.W, scene.H))
        for i in range(args.pretrain):
            pre.train_step(gt_images, directions, poses, allow_pair=i < args.pretrain - 1)
        pre.drain()
        torch.cuda.synchronize()
        transplant_state(pre, trainer)
        del pre
        torch.cuda.empty_cache()
    else:
        run(args.pretrain)
    torch.cuda.synchronize()
    log(rank, f"[bench] pretrain {args.pretrain} steps in {time.time() - t0:.1f}s, "
              f"samples last batch {int(trainer.n_samples.item())}")
    # ---- breakdown region: graph replays whose graphs carry HIP events
    # around every kernel (ktimer: external event nodes, read back one ring
    # slot behind); per-kernel durations of the step as it runs in the graphs
    n_bd = max(1, args.breakdown_steps)
    full = KT.KernelTimer(trainer.dctr, rows=max(4096, 2 * n_bd))
    trainer.timer = full
    run(64)  # capture this timer's graph variants
    torch.cuda.synchronize()
    full.reset()
    trainer.reset_stats()
    s_bd = adam_steps()
    t_bd = time.perf_counter()
    run(n_bd)
    torch.cuda.synchronize()
    t_bd = (time.perf_counter() - t_bd) / n_bd
    ran_bd = adam_steps() - s_bd
    trainer.timer = None
    bd_summary, bd_steps, bd_timeline = full.summary(), full.steps(), full.timeline()
    marched_bd, composited_bd, active_bd, evaluated_bd = trainer.stat_totals()
    if trainer.chunk_first <= 0:
        evaluated_bd = marched_bd
    fused_p = trainer.fused_params()
    pw = {"params": trainer.params.numel(), "fused_params": fused_p, "adam_params": trainer.params.numel() - fused_p}
    nb = max(1, ran_bd)  # (== n_bd: run() runs exactly n steps)
    units_bd = {"marched": marched_bd / nb, "evaluated": evaluated_bd / nb, "composited": composited_bd / nb,
                "active": active_bd / nb, **pw}

    def op_row(name, summary, units):
        """summary: {probe: (avg ms per launch, launches counted)}; every
        member is launched once per step in the rows counted"""
        bound, terms, members = WORK[name]
        ms = sum(summary[m][0] for m in members if m in summary)  # per step
        if ms <= 0:
            return None
        work = sum(units[basis] * per_unit for per_unit, basis in terms)  # per step
        peak, unit = PEAK[bound]
        achieved = work / (ms * 1e-3) / (1e9 if unit == "GB/s" else 1e12)
        return {"bound": bound, "achieved": round(achieved, 2), "peak": peak, "unit": unit,
                "frac": round(achieved / peak, 4), "ms_per_step": round(ms, 4),
                "work_per_step": round(work), "work_terms": [[pu, b, round(units[b], 1)] for pu, b in terms if units[b]],
                "kernels": members, "kernel_ms": {m: round(summary[m][0], 4) for m in members if m in summary},
                "launches_timed": min((summary[m][1] for m in members if m in summary), default=0)}

    kernels = {k: {"avg_launch_ms": round(v[0], 4), "launches_per_step": round(v[1], 2),
                   "ms_per_step": round(v[0] * v[1], 4)} for k, v in sorted(bd_summary.items(), key=lambda kv: -kv[1][0] * kv[1][1])}
    # ---- timed region: plain graph replays (no instrumentation: even two
    # stamp kernels per step cost ~3 %)
    run(args.warmup)
    torch.cuda.synchronize()
    trainer.reset_stats()
    s_timed = adam_steps()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    run(args.steps)
    t_enq = time.perf_counter() - t_start  # host time to enqueue the steps
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t_el = time.perf_counter() - t_start
    ran_timed = adam_steps() - s_timed
    if ran_timed != args.steps:
        raise RuntimeError(f"timed window ran {ran_timed} steps, expected {args.steps}")
    marched, composited, active, evaluated = trainer.stat_totals()
    # ---- roofline region: the same number of steps again, replaying the SAME
    # graphs as the timed window with the device probes armed (ktimer.ProbeTimer:
    # each probed kernel's execution span, no extra graph node); the steps that
    # open with an occupancy update (which launches field / march kernels a
    # second time in that step's row) are left out
    n_rf = min(args.steps, 32)  # (one probe row per step: 335 MB of slots)
    probes = KT.ProbeTimer(trainer.dctr, rows=n_rf)
    trainer.reset_stats()
    s_rf = adam_steps()
    probes.arm()
    vren._ok(vren.lib().ngp_trace_marker(1, vren._stream()), "trace_marker")  # window start (kernel traces)
    t_rf = time.perf_counter()
    run(n_rf)
    vren._ok(vren.lib().ngp_trace_marker(2, vren._stream()), "trace_marker")  # window end
    torch.cuda.synchronize()
    t_rf = (time.perf_counter() - t_rf) / n_rf
    probes.disarm()
    ran_rf = adam_steps() - s_rf
    ui = trainer.update_interval
    # (rows hold step % rows; a step whose number is a multiple of the update interval opens with
    # an occupancy update)
    skip = [r for r in range(probes.rows) if any(st % ui == 0 for st in range(s_rf, s_rf + ran_rf)
                                                 if st % probes.rows == r)]
    pr_summary = probes.summary(skip_rows=skip)
    pr_timeline = probes.timeline(skip_rows=skip)
    upd_steps = [st for st in range(s_rf, s_rf + ran_rf) if st % ui == 0]
    pr_gaps = probes.step_gaps(s_rf, ran_rf, skip_steps=upd_steps)
    m_rf, c_rf, a_rf, e_rf = trainer.stat_totals()
    # ---- the 1-in-update_interval step: a window of 4 update intervals with the probes armed (its own
    # rows: one per step); a step's period (its first kernel to the next step's first kernel) holds the
    # occupancy update and the next batch's march when an update follows it, against the median regular
    # period
    n_up = 4 * ui
    pu = KT.ProbeTimer(trainer.dctr, rows=n_up)
    s_up = adam_steps()
    pu.arm()
    run(n_up)
    torch.cuda.synchronize()
    pu.disarm()
    periods = pu.step_periods(s_up, adam_steps() - s_up)
    del pu
    p_upd = sorted(us for st, us in periods if (st + 1) % ui == 0)
    p_reg = sorted(us for st, us in periods if (st + 1) % ui != 0)
    update_step = None
    if p_upd and p_reg:
        reg, upd = p_reg[len(p_reg) // 2], p_upd[len(p_upd) // 2]
        update_step = {"interval": ui, "period_us": upd, "regular_period_us": reg, "extra_us": round(upd - reg, 1),
                       "amortised_extra_us_per_step": round((upd - reg) / ui, 1), "update_step_periods_us": p_upd,
                       "measured": f"medians over a {n_up}-step window after the roofline window (device probes)"}
    if trainer.chunk_first <= 0:
        e_rf = m_rf
    nr = max(1, ran_rf)
    units_rf = {"marched": m_rf / nr, "evaluated": e_rf / nr, "composited": c_rf / nr, "active": a_rf / nr, **pw}
    ops = {k: r for k in WORK if (r := op_row(k, pr_summary, units_rf)) is not None}
    if "hash_encode" in ops:
        # the encode's real limit is the lane-gather issue rate: 4 loads per level on dense levels,
        # 4 + 1/4 on hashed ones; scripts/diag/gather_diag.py measured 265 G lane-gathers/s for
        # random 4-16 B gathers from an L2-resident table, 72 G/s from a 24 MB one
        # (profiles/r02/gather_microbench.json)
        sizes = list(trainer.grid.desc.sizes)[:trainer.grid.n_levels]
        n_hashed = sum(1 for z in sizes if z == 1 << trainer.grid.log2_T)
        per_sample = 4 * (len(sizes) - n_hashed) + 5 * n_hashed
        ge = units_rf["evaluated"] * per_sample / (ops["hash_encode"]["ms_per_step"] * 1e-3)
        ops["hash_encode"]["lane_gathers_per_sample"] = per_sample
        ops["hash_encode"]["G_lane_gathers_per_s"] = round(ge / 1e9, 1)
        ops["hash_encode"]["gather_peak_note"] = ("random-gather rate 265 G/s L2-resident, 72 G/s from a 24 MB "
                                                  "table (profiles/r02/gather_microbench.json)")
        ops["hash_encode"]["fused_mlp_forward_flop_per_sample"] = _MLP_FWD
    for k, r in ops.items():
        r["traffic"] = pmc_traffic(PMC_KEYS.get(k, []))
    dominant = max((k for k in ops if k != "mlp_fwd"), key=lambda k: ops[k]["ms_per_step"])
    t_max = torch.tensor([t_el], device=dev)
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    t_el = float(t_max.item())
    total_rays = R * args.steps * world
    value = total_rays / t_el
    if trainer.chunk_first <= 0:
        evaluated = marched
    units = {"marched": marched / args.steps, "evaluated": evaluated / args.steps,
             "composited": composited / args.steps, "active": active / args.steps, **pw}
    rm_s, vr_s, ev_s = units["marched"] / R, units["composited"] / R, units["evaluated"] / R
    # units per step of each window: every window's own counters over exactly its own steps
    # (the roofline's units and its probes cover the same replays).  Within a window the counts
    # must nest -- gradient-carrying <= field-evaluated <= marched, composited <= marched,
    # gradient-carrying <= composited + one per ray (the terminating sample); ACROSS windows they
    # differ with the training state: on this workload the per-step composited samples swing
    # ~1.7x with a ~35-step period (profiles/r04/units_drift.json), so windows of 20 steps see
    # different work per step and only their own units are valid for them
    units_check = {"steps_run": {"breakdown": ran_bd, "timed": ran_timed, "roofline": ran_rf}}
    wins = {"breakdown": units_bd, "timed": units, "roofline": units_rf}
    for basis in ("marched", "evaluated", "composited", "active"):
        units_check[f"{basis}_per_step"] = {k: round(w[basis], 1) for k, w in wins.items()}
    nested = all(w["active"] <= w["evaluated"] + 0.5 and w["evaluated"] <= w["marched"] + 0.5
                 and w["composited"] <= w["marched"] + 0.5 and w["active"] <= w["composited"] + R + 0.5
                 for w in wins.values())
    steps_ok = ran_rf == n_rf and ran_bd == n_bd and ran_timed == args.steps
    vals = [w["composited"] for w in wins.values() if w["composited"] > 0]
    units_check["drift_composited_max_over_min"] = round(max(vals) / min(vals), 3) if vals else None
    units_check["ok"] = bool(nested and steps_ok)
    if not units_check["ok"]:
        print(f"[bench] WARNING: a window's unit counts do not nest or its step count is off: {units_check}",
              file=sys.stderr)
    roof = dict(op=dominant, traffic_unit="bytes per step", **ops[dominant], units_check=units_check,
                measured=f"sum of the op's kernels' execution spans (earliest wave start to latest wave end, "
                         f"device probes inside the kernels, ktimer.ProbeTimer) averaged over the "
                         f"{ops[dominant]['launches_timed']} steps of a {n_rf}-step window of the same "
                         f"graph replays as the timed one, steps opening with an occupancy update left out "
                         f"({t_rf * 1e3:.4f} ms/step in that window); rocprofv3 kernel-trace durations of the "
                         f"same command: scripts/roofline_check.py")
    # step-level bound: every op's algorithmic bytes at HBM peak + MLP FLOPs at MFMA peak
    def op_work(k):
        return sum(units[b] * pu for pu, b in KERNEL_WORK[k][1])
    # (all ops' work, the fused MLP forward's FLOPs included)
    hbm_bytes = sum(op_work(k) for k in KERNEL_WORK if KERNEL_WORK[k][0] != "mfma")
    flops = sum(op_work(k) for k in KERNEL_WORK if KERNEL_WORK[k][0] == "mfma")  # (mlp_fwd: the fused forward's)
    bound_ms = hbm_bytes / 8000e9 * 1e3 + flops / 2500e12 * 1e3
    adam_ms = units["params"] * 34 / 8000e9 * 1e3
    step_bound = {"hbm_bytes_per_step": round(hbm_bytes), "mlp_flops_per_step": round(flops),
                  "ms_per_step_at_peak": round(bound_ms, 4), "rays_per_s_at_peak": round(R / (bound_ms * 1e-3)),
                  "adam_ms_at_peak": round(adam_ms, 4),
                  "step_fraction_of_bound": round(bound_ms / (t_el / args.steps * 1e3), 4),
                  "note": "sum of the ops' algorithmic work at HBM / MFMA peak, serial; dense FusedAdam alone "
                          "(34 B/param) costs adam_ms_at_peak per step. rays_per_s_at_peak is this design's "
                          "floor under exact FusedAdam semantics: the north_star's 1e8 rays/s lies above it "
                          "(DESIGN.md section 7)"}
    loss = float(trainer.out_loss.sum().item())
    psnr = psnr_eval(trainer, scene, args.psnr_views, args.psnr_res) if (rank == 0 and args.psnr_views > 0) else None
    infer = inference_bench(trainer, args.infer_res, args.infer_frames, world, rank) if args.infer_frames > 0 else None
    dropin = None
    if rank == 0 and world == 1 and args.dropin_steps > 0:
        dropin = dropin_bench(trainer, gt_images, directions, poses, R, args.dropin_steps)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(trainer, scene, gt_images, R)
    quality = None
    if rank == 0 and world == 1 and args.quality_steps > 0:
        sys.path.insert(0, os.path.join(ROOT, "scripts"))
        import quality_30k
        quality = quality_30k.run(steps=args.quality_steps)
    oracle_q = None
    if rank == 0 and world == 1 and not args.no_oracle_quality:
        oracle_q = oracle_quality()
    # capacity guards (ngp_guard_hits): a device count clamped to its buffer's capacity anywhere in
    # this run -- samples dropped -- would make the line's work smaller than the step's
    guard_hits = int(vren.lib().ngp_guard_hits())
    if guard_hits:
        print(f"[bench] WARNING: {guard_hits} capacity guard hits (a device count clamped: work truncated)",
              file=sys.stderr)
    ms_step = t_el / args.steps * 1e3
    if rank == 0:
        out = {
            "metric": BASELINE["metric"], "value": round(value, 1), "unit": "rays/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "fp16 field (MLP forward, backward and weight gradients on fp16 MFMA operands, fp32 accumulate) / fp32 march, composite, Adam",
            "data": "synthetic (analytic sphere+box scene, 100 views 800x800, Lego intrinsics; random-init weights "
                    f"trained {args.pretrain} setup steps)",
            "config": {"workload": (f"{'lego' if args.scale <= 0.5 else 'garden'}-shaped training step: {R} rays/rank, "
                                    f"scale {args.scale:g}, {trainer.cascades} x 128^3 grid, L=16 F=2 T=2^19 hash, "
                                    f"64-wide MLPs, raw loss, Adam lr 1e-2"),
                       "batch_rays_per_gpu": R, "global_batch_rays": R * world, "pretrain_steps": args.pretrain,
                       "rm_samples_per_ray": round(rm_s, 2), "vr_samples_per_ray": round(vr_s, 2),
                       "field_evaluated_per_ray": round(ev_s, 2),
                       "graphs": trainer.use_graphs,
                       "chunk_first": trainer.chunk_first,
                       "row_forward": trainer.row_forward if trainer._rows_fwd(trainer.chunk_first) else 0,
                       "march_fork": trainer.march_fork_point(),
                       "parallelism": f"dp{world}" + (f" (data-parallel step of world {args.emulate_dp} emulated: collectives as local copies)" if args.emulate_dp else ""), "last_loss": round(loss, 5),
                       "hash_backward": args.hash_backward, "bin_level_lo": trainer.bin_level_lo,
                       "bin_merge_hi": trainer.bin_merge_hi,
                       "steps_per_graph_replay": 2 if trainer.pair_steps and world == 1 and not args.emulate_dp else 1,
                       "erode": trainer.erode,
                       "test_psnr_synthetic": round(psnr, 2) if psnr is not None else None},
            "roofline": roof,
            "ops": ops,
            "kernels": kernels,
            "timeline_us": bd_timeline,
            "probe_timeline_us": pr_timeline,
            "probe_step_gaps_us": {"gaps": [g for _, g in pr_gaps],
                                   "mean": round(sum(g for _, g in pr_gaps) / max(1, len(pr_gaps)), 1),
                                   "note": "end of a step's counters_inc to the next step's round 1, per "
                                           "consecutive step pair inside the probe window (pairs touching a step "
                                           "with an occupancy update left out; two steps per graph replay: "
                                           "alternately inside a graph and across a replay boundary)"},
            "step_bound": step_bound,
            # the timed window's step time per unit of its own work (the work per step follows the
            # training state, so these compare runs whose windows landed on different phases)
            "ns_per_composited_sample": round(ms_step * 1e6 / max(units["composited"], 1e-9), 4),
            "ns_per_marched_sample": round(ms_step * 1e6 / max(units["marched"], 1e-9), 4),
            "guard_hits": guard_hits,
            "occupancy_update_step": update_step,
            "host_enqueue_ms_per_step": round(t_enq / args.steps * 1e3, 4),
            "breakdown_note": (f"ops / kernels: wall-clock stamps around every kernel inside the captured graphs "
                               f"over {bd_steps} replayed steps ({t_bd * 1e3:.3f} ms/step with all stamps); timeline_us: "
                               f"average [start, end] of each launch (kernel#slot) from the step's first stamp, all "
                               f"streams; roofline: see roofline.measured"),
            "cpu_baseline": cpu,
            "quality": quality,
            "quality_vs_fp32_oracle": oracle_q,
            "inference": infer,
            "dropin": dropin,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
