#!/usr/bin/env python3
"""The training march alone on the chip (diagnostic): after the bench's 2000
setup steps, ngp_march_train_slots (the wave-per-ray lattice walk + its scan)
replayed 20x per graph and timed, then once with the device probes armed for
the per-wave start / end statistics (one ray per wave).  The library is the
one vren loads (NGP_AMD_LIB selects an A/B build).
usage: march_alone.py [setup_steps=2000]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd")]
import torch  # noqa: E402

import ktimer as KT  # noqa: E402
import synthetic as S  # noqa: E402
import vren  # noqa: E402
from trainer import NGPTrainer, ctypes_float  # noqa: E402


def main():
    n_setup = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    dev = torch.device("cuda")
    scene = S.AnalyticScene(W=800, H=800, n_images=100, scale=0.5)
    gt = scene.gt_images(device=dev)
    dirs, poses = scene.directions.to(dev).contiguous(), scene.poses.to(dev).contiguous()
    tr = NGPTrainer(scale=0.5, batch_size=8192, device=dev)
    tr.mark_invisible_cells(scene.K, scene.poses, (scene.W, scene.H))
    for i in range(n_setup):
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

    launch()
    torch.cuda.synchronize()
    counts = m["counts"].clone()
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
    res = {"lib": os.environ.get("NGP_AMD_LIB", "tree"), "march_slots_us": round(e0.elapsed_time(e1) * 1e3 / 100, 1)}
    assert torch.equal(counts, m["counts"])
    pt = KT.ProbeTimer(tr.dctr, rows=1)
    pt.arm()
    launch()
    pt.disarm()
    b = pt.buf[0, KT.PROBES.index("march"), :R].cpu().double()
    t0 = float(b[:, 0][b[:, 0] > 0].min())
    st, en = (b[:, 0] - t0) * pt.tick_ns * 1e-3, (b[:, 1] - t0) * pt.tick_ns * 1e-3
    dur = en - st
    ne = counts > 0
    q = lambda x: [round(float(torch.quantile(x, v)), 1) for v in (0.5, 0.9, 0.99)] + [round(float(x.max()), 1)]  # noqa: E731
    res.update({"span_us": round(float(en.max()), 1), "dur_mean_us": round(float(dur.mean()), 2),
                "dur_p50_p90_p99_max": q(dur), "dur_nonempty_mean_us": round(float(dur[ne.cpu()].mean()), 2),
                "start_p50_p90_max": q(st)[:2] + [round(float(st.max()), 1)],
                "rays_nonempty": int(ne.sum()), "marched": int(counts.sum()),
                "counts_sha": int((counts.long() * torch.arange(1, R + 1, device=counts.device)).sum())})
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
