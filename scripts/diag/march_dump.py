#!/usr/bin/env python3
"""Steady-state training march, alone on the chip (diagnostic): after the bench's
2000 setup steps, the training march kernel (ngp_march_train_slots: the
wave-per-ray walk, without / with cell windows, NGP_MARCH_CELLS) replayed 20x
per graph and timed; the batch's rays, hits, noise, counts and the occupancy
bitfield dumped to gpurun_out/march_state.npz for the window statistics on
the CPU (scripts/diag/march_windows.py)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import synthetic as S  # noqa: E402
import vren  # noqa: E402
from trainer import NGPTrainer, ctypes_float  # noqa: E402


def main():
    dev = torch.device("cuda")
    scene = S.AnalyticScene(W=800, H=800, n_images=100, scale=0.5)
    gt = scene.gt_images(device=dev)
    dirs, poses = scene.directions.to(dev).contiguous(), scene.poses.to(dev).contiguous()
    tr = NGPTrainer(scale=0.5, batch_size=8192, device=dev)
    tr.mark_invisible_cells(scene.K, scene.poses, (scene.W, scene.H))
    for _ in range(2000):
        tr.train_step(gt, dirs, poses)
    tr.drain()
    torch.cuda.synchronize()
    m = tr.msets[tr.cur]
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    R = tr.batch_size

    def launch():
        vren._ok(tr.L.ngp_march_train_slots(p(m["rays_o"]), p(m["rays_d"]), p(m["hits_t"]), R, p(tr.density_bitfield),
                                            tr.cascades, tr.G, ctypes_float(tr.scale), ctypes_float(tr.esf),
                                            p(m["noise"]), tr.max_samples, p(m["counts"]), p(m["rays_a"]),
                                            p(m["n_samples"]), p(m["slot_t"]), p(m["slot_dt"]), p(m["occ_summary"]),
                                            vren._stream()), "march_slots")

    res = {}
    counts = {}
    for cells in ("0", "1"):
        os.environ["NGP_MARCH_CELLS"] = cells
        launch()
        torch.cuda.synchronize()
        counts[cells] = m["counts"].clone()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(20):
                launch()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        res[f"march_slots_us_cells{cells}"] = round(e0.elapsed_time(e1) * 1e3 / 100, 1)
    # per-wave spans (device probes: lane 0 of each wave stores its start / end; one ray per wave)
    import ktimer as KT
    pt = KT.ProbeTimer(tr.dctr, rows=1)
    waves = {}
    for cells in ("0", "1"):
        os.environ["NGP_MARCH_CELLS"] = cells
        pt.arm()
        launch()
        pt.disarm()
        b = pt.buf[0, KT.PROBES.index("march"), :R].cpu().double()
        t0 = float(b[:, 0][b[:, 0] > 0].min())
        waves[cells] = ((b[:, 0] - t0) * pt.tick_ns * 1e-3, (b[:, 1] - t0) * pt.tick_ns * 1e-3)  # us
        st, en = waves[cells]
        dur = en - st
        res[f"waves_cells{cells}"] = {"span_us": round(float(en.max()), 1), "dur_mean_us": round(float(dur.mean()), 2),
                                      "dur_p50_p90_p99_max": [round(float(x), 1) for x in
                                                              np.percentile(dur.numpy(), [50, 90, 99, 100])],
                                      "start_p50_p90_max": [round(float(x), 1) for x in
                                                            np.percentile(st.numpy(), [50, 90, 100])]}
    res["counts_equal"] = bool(torch.equal(counts["0"], counts["1"]))
    c = counts["0"].cpu()
    res["rays"] = R
    res["rays_nonempty"] = int((c > 0).sum())
    res["marched"] = int(c.sum())
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", "march_state.npz"),
                        rays_o=m["rays_o"].cpu().numpy(), rays_d=m["rays_d"].cpu().numpy(),
                        hits_t=m["hits_t"].cpu().numpy(), noise=m["noise"].cpu().numpy(), counts=c.numpy(),
                        bitfield=tr.density_bitfield.cpu().numpy(),
                        **{f"wave_{k}_{j}": waves[k][j].numpy() for k in waves for j in (0, 1)})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
