"""Distribution of marched samples per ray and of composited (gradient-
carrying) samples per ray at training steady state: the composite kernel's
time is set by its longest rows."""
import json
import os
import sys

H = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(H, "..", ".."), os.path.join(H, "..", "..", "ar-nerf_amd")]
import torch  # noqa: E402

import synthetic as S  # noqa: E402
from trainer import NGPTrainer  # noqa: E402

dev = torch.device("cuda")
scene = S.AnalyticScene(W=800, H=800, n_images=100, scale=0.5)
gt = scene.gt_images(device=dev)
dirs, poses = scene.directions.to(dev), scene.poses.to(dev)
tr = NGPTrainer(scale=0.5, batch_size=8192, device=dev, use_graphs=False)
tr.mark_invisible_cells(scene.K, scene.poses, (scene.W, scene.H))
# (eager steps: the trainer is built with use_graphs=False below)
for _ in range(2000):
    tr.train_step(gt, dirs, poses)
tr.drain()
torch.cuda.synchronize()
tr.use_graphs = False
tr.train_step(gt, dirs, poses)
torch.cuda.synchronize()
N = tr.rays_a[:, 2].float().cpu()
A = tr.n_active.float().cpu()
q = torch.tensor([0.5, 0.9, 0.99, 0.999, 1.0])
out = {"marched_quantiles": torch.quantile(N, q).tolist(), "active_quantiles": torch.quantile(A, q).tolist(),
       "rows_over_128": int((N > 128).sum()), "rows_over_256": int((N > 256).sum()),
       "active_over_64": int((A > 64).sum()), "not_terminated": int((A >= N).sum())}
print(json.dumps(out))
