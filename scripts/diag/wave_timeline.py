#!/usr/bin/env python3
"""Per-wave timeline of the graph-replayed training step (diagnostic): the
device probes (lane 0 of every wave of a probed kernel stores its start and
end) of a few steady-state steps; per kernel: first start / last end, wave
start and duration quantiles, and the number of its waves running at each
4-us point of the step -- whether a kernel beside the march waits to START
its waves (residency) or runs them slowly (issue).
usage: wave_timeline.py [steps=4]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ktimer as KT  # noqa: E402
import synthetic as S  # noqa: E402
from trainer import NGPTrainer  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
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
    pt = KT.ProbeTimer(tr.dctr, rows=16)
    pt.arm()
    run(16)
    pt.disarm()
    b = pt.buf.cpu().numpy().astype(np.float64) * pt.tick_ns * 1e-3  # us
    out = {}
    rows = []
    for r in range(16):
        fc = b[r, KT.PROBES.index("first_chunk")]
        if not (fc[:, 0] > 0).any() or not (b[r, KT.PROBES.index("march"), :, 0] > 0).any():
            continue
        rows.append(r)
    for r in rows[:n]:
        t0 = b[r, KT.PROBES.index("first_chunk")][:, 0]
        t0 = t0[t0 > 0].min()
        step = {}
        for k, name in enumerate(KT.PROBES):
            w = b[r, k]
            m = w[:, 0] > 0
            if not m.any():
                continue
            st, en = w[m, 0] - t0, w[m, 1] - t0
            conc = [int(((st <= x) & (en > x)).sum()) for x in np.arange(0, 500, 4)]
            step[name] = {"waves": int(m.sum()), "first_start": round(float(st.min()), 1),
                          "last_end": round(float(en.max()), 1),
                          "start_q10_50_90": [round(float(x), 1) for x in np.percentile(st, [10, 50, 90])],
                          "dur_q10_50_90": [round(float(x), 1) for x in np.percentile(en - st, [10, 50, 90])],
                          "running_every_4us": conc}
        out[f"row{r}"] = step
    for r, step in out.items():
        print(r)
        for name, v in sorted(step.items(), key=lambda kv: kv[1]["first_start"]):
            c = v["running_every_4us"]
            lo, hi = int(v["first_start"] // 4), int(v["last_end"] // 4) + 1
            print(f"  {name:18s} waves {v['waves']:6d} [{v['first_start']:7.1f}, {v['last_end']:7.1f}] start q10/50/90 "
                  f"{v['start_q10_50_90']} dur q10/50/90 {v['dur_q10_50_90']} running: {c[max(lo, 0):min(hi, len(c))]}")
    with open(os.path.join(ROOT, "gpurun_out", "wave_timeline.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
