#!/usr/bin/env python3
"""What each side branch of the graph-replayed training step costs the critical
path (diagnostic, NOT a valid training run): after the bench's setup training,
the step is re-captured with one branch left out and timed against the full
step, alternating.  Variants:
  full      the product step
  nomarch   the next batch's march (side stream) left out: the step re-uses
            a batch marched earlier (identical work shape, stale batch)
  nocoarse  the atomic coarse hash levels left out (their Adam still runs)
  neither   both left out
usage: skip_cost.py [steps_per_window=300] [rounds=3]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd")]
import torch  # noqa: E402

import synthetic as S  # noqa: E402
from trainer import NGPTrainer  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda")
    scene = S.AnalyticScene(W=800, H=800, n_images=100, scale=0.5)
    gt = scene.gt_images(device=dev)
    dirs, poses = scene.directions.to(dev).contiguous(), scene.poses.to(dev).contiguous()
    tr = NGPTrainer(scale=0.5, batch_size=8192, device=dev, pair_steps=True)
    tr.mark_invisible_cells(scene.K, scene.poses, (scene.W, scene.H))

    def run(k):
        for i in range(k):
            tr.train_step(gt, dirs, poses, allow_pair=i < k - 1)
        tr.drain()

    run(2000)
    torch.cuda.synchronize()
    march0, coarse0 = tr._march, tr._coarse_levels
    L0 = tr.L
    side = tr.march_stream.cuda_stream

    class LProxy:
        """the library with chosen launches of the side stream's march left out"""
        skip = ()

        def __getattr__(self, k):
            f = getattr(L0, k)
            if k not in self.skip:
                return f

            def g(*a):
                s = a[-1]
                if (s.value if hasattr(s, "value") else s) == side:
                    return 0
                return f(*a)
            return g

    names = sys.argv[3].split(",") if len(sys.argv) > 3 else ["full", "nomarch", "nocoarse", "neither"]
    # (only launches whose outputs stay consistent when left out: without the march kernel + its scan
    # the set keeps an earlier batch's counts, rays_a and slots, which the compaction then re-reads)
    skips = {"nomarchkernel": ("ngp_march_train_slots",)}

    def variant(name):
        skip_m = name in ("nomarch", "neither")
        skip_c = name in ("nocoarse", "neither")
        if name in skips:
            px = LProxy()
            px.skip = skips[name]
            tr.L = px
        else:
            tr.L = L0

        def march(k, src, directions, poses, stream):
            if skip_m and stream is tr.march_stream:
                # the set's round-2 list counter is reset by the march's rays_nonempty launch:
                # without it the row forward's reservations would run past the list
                with torch.cuda.stream(stream):
                    tr.msets[k]["eval_total2"].zero_()
                return None
            return march0(k, src, directions, poses, stream)

        tr._march = march
        tr._coarse_levels = (lambda fold=True: None) if skip_c else coarse0
        tr._graphs = {}
        run(64)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(n)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e6

    res = {}
    for r in range(rounds):
        for name in names:
            us = variant(name)
            res.setdefault(name, []).append(round(us, 1))
            print(name, r, round(us, 1), "us/step", flush=True)
    tr._march, tr._coarse_levels, tr.L = march0, coarse0, L0
    # the training march alone on the chip (sample_batch .. rays_nonempty), 20 per graph
    cs = torch.cuda.current_stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20):
            march0(tr.cur, ("sample", 1, gt), dirs, poses, torch.cuda.current_stream())
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(cs)
    for _ in range(5):
        g.replay()
    e1.record(cs)
    torch.cuda.synchronize()
    res["march_alone_us"] = round(e0.elapsed_time(e1) * 1e3 / 100, 1)
    print(json.dumps({k: ({"us": v, "mean": round(sum(v) / len(v), 1)} if isinstance(v, list) else v)
                      for k, v in res.items()}))


if __name__ == "__main__":
    main()
