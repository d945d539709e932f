"""Per-step sample counts of the bench's training run (diagnostic): after the
bench's 2000 pretrain steps, 400 more graph-replayed steps (one step per
replay), each followed by a synchronize and a read of the step's marched /
composited / gradient-carrying / evaluated counts -- how much these units
move from one 20-step window to the next (the roofline's units come from its
own window).  Prints one JSON line: per-20-step-window means and the per-step
series of composited samples."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd")]

import torch  # noqa: E402

import synthetic as S  # noqa: E402
from trainer import NGPTrainer  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
sc = S.AnalyticScene(W=800, H=800, n_images=100, scale=0.5)
gt = sc.gt_images(device=dev)
dirs, poses = sc.directions.to(dev).contiguous(), sc.poses.to(dev).contiguous()
tr = NGPTrainer(scale=0.5, batch_size=8192, device=dev)
tr.mark_invisible_cells(sc.K, sc.poses, (sc.W, sc.H))
for _ in range(2000):
    tr.train_step(gt, dirs, poses)
tr.drain()
torch.cuda.synchronize()
rows = []
for i in range(400):
    tr.reset_stats()
    loss = tr.train_step(gt, dirs, poses)
    tr.drain()
    torch.cuda.synchronize()
    m, c, a, e = tr.stat_totals()
    rows.append((m, c, a, e, float(loss.mean())))
wins = []
for w in range(0, 400, 20):
    seg = rows[w:w + 20]
    wins.append([round(sum(r[k] for r in seg) / len(seg)) for k in range(4)] + [sum(r[4] for r in seg) / len(seg)])
print(json.dumps({"windows_20_steps_marched_composited_active_evaluated_loss": wins,
                  "composited_per_step": [r[1] for r in rows]}))
