"""Time NGPTrainer.update_density_grid (sampled, eager) with and without the
kept-sample evaluation (occ_keep), after a short training run; per-kernel
times from a torch profiler pass.  usage: python scripts/diag/occ_keep_time.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import synthetic as S  # noqa: E402
from trainer import NGPTrainer  # noqa: E402

THR = 0.01 * 1024 / 3 ** 0.5
sc = S.AnalyticScene(W=200, H=200, n_images=20)
dirs, poses = sc.directions.cuda(), sc.poses.cuda()
gt = sc.gt_images(device="cuda")
tr = NGPTrainer(scale=0.5, batch_size=8192, device="cuda", seed=3, warmup_steps=256)
tr.mark_invisible_cells(sc.K, sc.poses, (sc.W, sc.H))
for _ in range(600):
    tr.train_step(gt, dirs, poses)
tr.drain()
torch.cuda.synchronize()
for keep in (False, True, False, True):
    tr.occ_keep = keep
    for _ in range(3):
        tr.update_density_grid(THR, warmup=False)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        tr.update_density_grid(THR, warmup=False)
    b.record()
    torch.cuda.synchronize()
    print(f"keep={keep}: {a.elapsed_time(b) / 20 * 1e3:.1f} us per update; kept {int(tr._occ_kept_n.item())}")
for keep in (False, True):
    tr.occ_keep = keep
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        for _ in range(10):
            tr.update_density_grid(THR, warmup=False)
        torch.cuda.synchronize()
    print(f"keep={keep}")
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=14))
