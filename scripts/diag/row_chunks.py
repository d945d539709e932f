"""Per-row work of the chunked forward (diagnostic): after the bench's 2000
pretrain steps, several batches' rays_a / deltas and the density of EVERY
marched sample (one field launch over the whole march), then on the host:
marched samples per row, the samples the two-round chunked forward evaluates
(first 64 of each row + the whole rest of rows still transparent after them),
the samples a per-row loop over 64-sample chunks evaluates (stop after the
chunk in which the row's transmittance falls below 1e-4), and the lane slots
a one-row-per-wave loop would occupy.  Prints one JSON line."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd")]

import torch  # noqa: E402

import hashgrid as HG  # noqa: E402
import synthetic as S  # noqa: E402
import vren  # noqa: E402
from trainer import NGPTrainer, _p  # noqa: E402

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
print("pretrained", flush=True)
HGL = HG._lib()
K, thr = 64, 1e-4
agg = {"rows": 0, "rows_nonempty": 0, "marched": 0, "two_round": 0, "loop": 0, "loop_slots": 0,
       "round1": 0, "round2": 0, "rows_round2": 0}
hist_n = np.zeros(9, np.int64)  # N in [0], [1,16], (16,32], (32,48], (48,64], (64,128], (128,256], (256,512], >512
hist_chunks = np.zeros(8, np.int64)
for b in range(8):
    tr.train_step(gt, dirs, poses)
    tr.drain()
    torch.cuda.synchronize()
    m = tr.msets[tr.cur]
    ns = int(m["n_samples"][0])
    sig = torch.zeros(tr.cap, dtype=torch.float32, device=dev)
    rgb = torch.zeros(tr.cap * 3, dtype=torch.float32, device=dev)
    vren._ok(HGL.ngp_field_encode_mlp(_p(m["xyzs"]), _p(m["dirs"]), tr.cap, _p(m["n_samples"]), None,
                                      HG.ctypes.byref(tr.grid.desc), _p(tr.params16[HG.MLP_PARAMS:]),
                                      _p(tr.params16), None, _p(sig), _p(rgb), None, vren._stream()), "field")
    torch.cuda.synchronize()
    ra = m["rays_a"].view(-1, 3).cpu().numpy()
    s = sig[:ns].cpu().numpy().astype(np.float64)
    d = m["deltas"][:ns].cpu().numpy().astype(np.float64)
    a = 1.0 - np.exp(-s * d)
    for r in range(ra.shape[0]):
        st, N = int(ra[r, 1]), int(ra[r, 2])
        agg["rows"] += 1
        agg["marched"] += N
        hist_n[np.searchsorted([0, 16, 32, 48, 64, 128, 256, 512], N, side="left")] += 1
        if N == 0:
            continue
        agg["rows_nonempty"] += 1
        T = np.cumprod(1.0 - a[st:st + N])
        hit = np.nonzero(T < thr)[0]
        term = int(hit[0]) if hit.size else N  # index of the sample at which T falls below thr
        r1 = min(N, K)
        agg["round1"] += r1
        if term >= K and N > K:
            agg["round2"] += N - K
            agg["rows_round2"] += 1
        agg["two_round"] += r1 + (N - K if (term >= K and N > K) else 0)
        nch = min((N + 63) // 64, term // 64 + 1)
        agg["loop"] += min(N, 64 * nch)
        agg["loop_slots"] += 64 * nch
        hist_chunks[min(nch, 7)] += 1
agg["hist_marched_per_row_edges"] = "0 | 1-16 | 17-32 | 33-48 | 49-64 | 65-128 | 129-256 | 257-512 | >512"
agg["hist_marched_per_row"] = hist_n.tolist()
agg["hist_loop_chunks_per_row"] = hist_chunks.tolist()
agg["loop_lane_utilisation"] = round(agg["loop"] / max(1, agg["loop_slots"]), 3)
agg["batches"] = 8
print(json.dumps(agg))
