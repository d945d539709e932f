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

import hashgrid as HG  # noqa: E402
import synthetic as S  # noqa: E402
from trainer import NGPTrainer  # noqa: E402

with open(os.path.join(ROOT, "BASELINE.json")) as f:
    BASELINE = json.load(f)

# Algorithmic work per unit of the per-kernel breakdown:
#  hash_encode (unit: field-evaluated sample): 16 levels x 8 corners x fp16x2
#      gathered (512 B) + xyz (12 B) + list index (4 B) read + fp16 encoding
#      (64 B) written                                              -> bytes
#  field_mlp (evaluated sample): density 32-64-16 + colour 32-64-64-16 forward
#      (2 x (3072 + 7168) FLOP)                                    -> FLOPs
#  mlp_bwd (gradient-carrying sample): forward recompute + dX + dW of both
#      MLPs (16-row output layers as computed)                     -> FLOPs
#  hash_bwd_coarse (gradient-carrying sample, levels 0-7): xyz + index (16 B)
#      + dL/denc (64 B) read + read-modify-write of 8 x 8 x 2 fp32 table
#      gradients (2 x 512 B)                                       -> bytes
#  adam (parameter): p, g, m, v read; p, m, v, fp16 p written, g zeroed (34 B)
_MLP_FWD = 2 * (32 * 64 + 64 * 16) + 2 * (32 * 64 + 64 * 64 + 64 * 16)
KERNEL_WORK = {
    "hash_encode": ("hbm", 16 * 8 * 4 + 12 + 4 + 64, "GB/s", "evaluated"),
    "field_mlp": ("mfma", _MLP_FWD, "TFLOP/s", "evaluated"),
    "mlp_bwd": ("mfma", 2 * (32 * 64 + 64 * 16 + 32 * 64 + 64 * 64 + 64 * 16)
                + 2 * (16 * 64 + 64 * 64 + 64 * 16 + 16 * 64 + 64 * 32)
                + 2 * (16 * 64 + 64 * 64 + 64 * 32 + 16 * 64 + 64 * 32), "TFLOP/s", "active"),
    "hash_bwd_coarse": ("hbm", 16 + 64 + 2 * 8 * 8 * 2 * 4, "GB/s", "active"),
    "adam": ("hbm", 34, "GB/s", "params"),
}
PEAK = {"hbm": 8000.0, "mfma": 2500.0}  # MI355X: HBM3E GB/s; dense fp16 MFMA TFLOP/s


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
    ap.add_argument("--cpu-budget-s", type=float, default=15.0)
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--breakdown-steps", type=int, default=50, help="eager steps with per-kernel HIP events")
    ap.add_argument("--hash-backward", default="hybrid", choices=["hybrid", "binned", "atomic"])
    ap.add_argument("--bin-level-lo", type=int, default=None,
                    help="hybrid hash backward: first binned level (default: trainer's, 8 / 0 for cascaded scenes)")
    ap.add_argument("--bin-samples-per-ray", type=int, default=None,
                    help="binned hash-backward workspace per ray (default: trainer's, 128 / 512 for cascaded scenes)")
    ap.add_argument("--erode", default="auto", choices=["auto", "on", "off"],
                    help="occupancy erode decay (networks.py:270-272); auto = on for cascaded (garden-shaped, "
                         "COLMAP-like) scenes as train.py:178 does for colmap")
    ap.add_argument("--infer-frames", type=int, default=20, help="timed full-frame test renders (0: skip)")
    ap.add_argument("--infer-res", type=int, default=800)
    return ap.parse_args()


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, local


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


def inference_bench(trainer, res, frames, world, rank):
    """BASELINE config 5: full-frame test-time render (models/rendering.py:162-253)
    of the trained model, graph-captured (renderer.TestRenderer), `frames` poses
    per rank (frames are independent: replicas).  The host-driven loop
    (trainer.render, the reference's control flow) is timed on one frame beside it."""
    import renderer as RD
    sc = S.AnalyticScene(W=res, H=res, n_images=max(2, frames), scale=trainer.scale, seed=321 + rank)
    n = res * res
    rr = RD.TestRenderer(n, trainer.grid, trainer.params16, trainer.density_bitfield, trainer.cascades,
                         trainer.scale, trainer.G, exp_step_factor=trainer.esf, iters_per_graph=16, iters_tail=8)
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
            "host_loop_ms_per_frame": round(t_host * 1e3, 3), "host_loop_bit_exact": same,
            "workload": "full-frame test render of the trained model (black bg), march+field+composite per "
                        "iteration in HIP graphs (16 iterations, then 8 per replay while rays remain), one host sync per graph"}


def cpu_baseline(trainer, scene, gt_images, budget_s, batch):
    """The oracle (oracle/, CPU restatement) timed on this host on the same
    workload: full training steps on 8192-ray batches from the same model
    state, as many as fit ~budget_s (at least 1)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # test/baseline infrastructure only
    threads = int(os.environ.get("OMP_NUM_THREADS", min(16, os.cpu_count() or 1)))
    torch.set_num_threads(threads)
    ot = O.OracleTrainer(trainer.params, scene.scale, trainer.density_bitfield, trainer.cascades)
    gen = torch.Generator().manual_seed(77)
    c = torch.zeros(1, 3); h = torch.ones(1, 3) * scene.scale
    steps, t_total, samples = 0, 0.0, 0
    while steps < 5 and (steps == 0 or t_total < budget_s):
        img, pix = scene.sample_batch(batch, gen)
        o, d = scene.rays(img, pix)
        _, ht, _ = O.ray_aabb_intersect(o, d, c, h, 1)
        ht = ht[:, 0].contiguous()
        ht[(ht[:, 0] >= 0) & (ht[:, 0] < 0.01), 0] = 0.01
        gt = gt_images[img, pix].float().cpu() / 255
        noise = torch.rand(batch, generator=gen)
        t0 = time.perf_counter()
        _, n = ot.step(o.contiguous(), d.contiguous(), ht, gt, noise, torch.ones(3))
        t_total += time.perf_counter() - t0
        steps += 1
        samples += n
    return {"value": round(batch * steps / t_total, 1), "unit": "rays/s", "cores": threads, "kind": "port",
            "sample": f"{steps} full training step(s) of the {batch}-ray batch on the oracle "
                      f"(C march/composite/hash + torch fp32 MLP autograd + C Adam over all params), "
                      f"{samples / max(1, steps) / batch:.1f} samples/ray, {t_total:.1f} s"}


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed PMC summary
    (profiles/pmc_traffic.json, written by scripts/pmc_traffic.py from
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this bench,
    corrected per MI355X_MICROARCH.md "HBM"), or None if not measured."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            t = json.load(f).get(kernel)
    except (OSError, ValueError):
        return None
    return None if t is None else t.get("bytes_per_launch")


def _recorded(event):
    try:
        event.elapsed_time(event)
        return True
    except (RuntimeError, ValueError):
        return False


def main():
    args = parse()
    world, rank, local = setup_dist(args)
    dev = torch.device("cuda", local)
    torch.manual_seed(0)
    scene = S.AnalyticScene(W=args.res, H=args.res, n_images=args.images, scale=args.scale)
    gt_images = scene.gt_images(device=dev)  # (n_img, HW, 3) u8, resident in HBM
    directions = scene.directions.to(dev).contiguous()
    poses = scene.poses.to(dev).contiguous()
    erode = args.erode == "on" or (args.erode == "auto" and args.scale > 0.5)
    trainer = NGPTrainer(scale=args.scale, batch_size=args.batch, device=dev, hash_backward=args.hash_backward,
                         bin_level_lo=args.bin_level_lo, bin_samples_per_ray=args.bin_samples_per_ray, erode=erode)
    trainer.mark_invisible_cells(scene.K, scene.poses, (scene.W, scene.H))
    R = args.batch

    def run(n, events=None):
        """n training steps, each on a batch drawn on device (trainer.train_step:
        pixels, ground truth and noise from a counter-based RNG); batch i+1 is
        drawn and marched on the side stream during step i."""
        for i in range(n):
            if events is not None:
                trainer.kernel_events = events[i]
            trainer.train_step(gt_images, directions, poses)
        trainer.drain()

    t0 = time.time()
    run(args.pretrain)
    torch.cuda.synchronize()
    log(rank, f"[bench] pretrain {args.pretrain} steps in {time.time() - t0:.1f}s, "
              f"samples last batch {int(trainer.n_samples.item())}")
    run(args.warmup)
    # ---- timed region: steady-state steps replay captured HIP graphs
    # (trainer.train_step); no per-kernel instrumentation inside
    trainer.stats.zero_()
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
    t_max = torch.tensor([t_el], device=dev)
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    t_el = float(t_max.item())
    total_rays = R * args.steps * world
    value = total_rays / t_el
    marched, composited, active, evaluated = trainer.stat_totals()
    if trainer.chunk_first <= 0:
        evaluated = marched
    rm_s = marched / (R * args.steps)
    vr_s = composited / (R * args.steps)
    ev_s = evaluated / (R * args.steps)
    # ---- breakdown region: the same steps run eagerly with HIP events around
    # each kernel / stage, on the stream each is launched on (events cannot
    # sit between the nodes of a replayed graph); per-kernel durations and the
    # roofline come from here
    n_bd = max(1, min(args.steps, args.breakdown_steps))
    # raygen_march = inline march on the main stream (steps after an occupancy
    # update); march_side = the next batch's march on the side stream, which
    # overlaps the step's compute (averaged over the steps that launched one)
    stages = ["occupancy_update", "raygen_march", "march_side", "field_fwd", "composite_loss", "composite", "mlp_bwd",
              "hash_bwd",
              "hash_binned_apply", "allreduce", "adam"]
    ev = [dict() for _ in range(n_bd)]
    trainer.stats.zero_()
    torch.cuda.synchronize()
    t_bd = time.perf_counter()
    run(n_bd, ev)
    torch.cuda.synchronize()
    t_bd = time.perf_counter() - t_bd
    trainer.kernel_events = None
    marched_bd, _, active_bd, evaluated_bd = trainer.stat_totals()
    if trainer.chunk_first <= 0:
        evaluated_bd = marched_bd

    def durations(name):
        return [p[0].elapsed_time(p[1]) for e in ev for p in e.get(name, []) if _recorded(p[1])]

    per_step = {"evaluated": evaluated_bd / n_bd, "active": active_bd / n_bd, "params": trainer.params.numel()}
    kernels = {}
    for k, (bound, per_unit, unit, basis) in KERNEL_WORK.items():
        d = durations(k)
        if not d:
            continue
        ms = sum(d) / len(d)
        launches = len(d) / n_bd
        units = per_step[basis] / launches if basis != "params" else per_step[basis] / launches
        achieved = units * per_unit / (ms * 1e-3) / (1e9 if bound == "hbm" else 1e12)
        kernels[k] = {"bound": bound, "achieved": round(achieved, 2), "peak": PEAK[bound], "unit": unit,
                      "frac": round(achieved / PEAK[bound], 4), "avg_launch_ms": round(ms, 4),
                      "launches_per_step": round(launches, 2), "work_per_unit": per_unit,
                      "units_per_launch": round(units, 1), "unit_basis": basis}
    dominant = max(kernels, key=lambda k: kernels[k]["avg_launch_ms"])
    stage_ms = {}
    for k in stages:
        d = durations(k)
        if d:  # per step (march_side: per launch, over the steps that launched one)
            stage_ms[k] = round(sum(d) / (len(d) if k == "march_side" else n_bd), 4)
    loss = float(trainer.out_loss.sum().item())
    psnr = psnr_eval(trainer, scene, args.psnr_views, args.psnr_res) if (rank == 0 and args.psnr_views > 0) else None
    infer = inference_bench(trainer, args.infer_res, args.infer_frames, world, rank) if args.infer_frames > 0 else None
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(trainer, scene, gt_images, args.cpu_budget_s, R)
    if rank == 0:
        out = {
            "metric": BASELINE["metric"], "value": round(value, 1), "unit": "rays/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(t_el / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp16/fp32",
            "data": "synthetic (analytic sphere+box scene, 100 views 800x800, Lego intrinsics; random-init weights "
                    f"trained {args.pretrain} setup steps)",
            "config": {"workload": "lego-shaped training step: 8192 rays/rank, scale 0.5, 128^3 grid, L=16 F=2 "
                                   "T=2^19 hash, 64-wide MLPs, raw loss, Adam lr 1e-2",
                       "batch_rays_per_gpu": R, "global_batch_rays": R * world, "pretrain_steps": args.pretrain,
                       "rm_samples_per_ray": round(rm_s, 2), "vr_samples_per_ray": round(vr_s, 2),
                       "field_evaluated_per_ray": round(ev_s, 2),
                       "graphs": trainer.use_graphs,
                       "chunk_first": trainer.chunk_first,
                       "parallelism": f"dp{world}", "last_loss": round(loss, 5),
                       "hash_backward": args.hash_backward, "bin_level_lo": trainer.bin_level_lo,
                       "erode": trainer.erode,
                       "test_psnr_synthetic": round(psnr, 2) if psnr is not None else None},
            "roofline": dict(kernel=dominant, traffic=pmc_traffic(dominant), **kernels[dominant]),
            "kernels": kernels,
            "stage_ms": stage_ms,
            "host_enqueue_ms_per_step": round(t_enq / args.steps * 1e3, 4),
            "breakdown_note": (f"kernels / stage_ms / roofline: HIP-event averages over {n_bd} eagerly run steps after "
                               f"the timed region ({t_bd / n_bd * 1e3:.3f} ms/step eager); the timed steps replay "
                               "captured HIP graphs"),
            "cpu_baseline": cpu,
            "inference": infer,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
