#!/usr/bin/env python3
"""Training march variants on ONE batch (diagnostic): after setup training
with the tree's library, the same ray batch / bitfield is marched by the
ngp_march_train_slots of every library given (each loaded under its own
path: A/B builds side by side in one process) -- per library: kernel time
(20 launches per graph replay), per-wave start / end from its device probes,
and the per-ray counts checked equal to the tree's (bit-exact slots too).
usage: march_libs.py SETUP_STEPS LIB.so [LIB.so ...]"""
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
from trainer import NGPTrainer  # noqa: E402

vp = ctypes.c_void_p


def declare(L):
    L.ngp_march_train_slots.argtypes = [vp, vp, vp, ctypes.c_int64, vp, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                        ctypes.c_float, vp, ctypes.c_int, vp, vp, vp, vp, vp, vp, vp]
    L.ngp_march_train_slots.restype = ctypes.c_int
    L.ngp_probe_set.argtypes = [vp, vp, ctypes.c_int64]
    L.ngp_probe_set.restype = ctypes.c_int
    return L


def main():
    n_setup = int(sys.argv[1])
    libs = sys.argv[2:]
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
    R = tr.batch_size
    p = lambda t: vp(t.data_ptr())  # noqa: E731
    outs = {}
    probe_buf = torch.zeros(1, len(KT.PROBES), KT.ProbeTimer.WAVES, 2, dtype=torch.int64, device=dev)
    step0 = torch.zeros(1, dtype=torch.int64, device=dev)
    tick = vren.lib().ngp_timing_tick_ns()
    for path in libs:
        L = declare(ctypes.CDLL(os.path.abspath(path)))
        counts = torch.empty(R, dtype=torch.int32, device=dev)
        rays_a = torch.empty(R, 3, dtype=torch.int64, device=dev)
        tot = torch.zeros(1, dtype=torch.int64, device=dev)
        st, sd = torch.zeros_like(m["slot_t"]), torch.zeros_like(m["slot_dt"])

        def launch():
            r = L.ngp_march_train_slots(p(m["rays_o"]), p(m["rays_d"]), p(m["hits_t"]), R, p(tr.density_bitfield),
                                        tr.cascades, tr.G, tr.scale, tr.esf, p(m["noise"]), tr.max_samples, p(counts),
                                        p(rays_a), p(tot), p(st), p(sd), p(m["occ_summary"]),
                                        vp(torch.cuda.current_stream().cuda_stream))
            assert r == 0, r
        launch()
        torch.cuda.synchronize()
        c0, s0, d0 = counts.clone(), st.clone(), sd.clone()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(20):
                launch()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 200
        probe_buf.zero_()
        assert L.ngp_probe_set(p(probe_buf), p(step0), 1) == 0
        launch()
        torch.cuda.synchronize()
        assert L.ngp_probe_set(None, None, 0) == 0
        b = probe_buf[0, KT.PROBES.index("march"), :R].cpu().double()
        t0 = float(b[:, 0][b[:, 0] > 0].min())
        sw, ew = (b[:, 0] - t0) * tick * 1e-3, (b[:, 1] - t0) * tick * 1e-3
        dur = ew - sw
        ne = (c0 > 0).cpu()
        q = lambda x: [round(float(torch.quantile(x, v)), 1) for v in (0.5, 0.9, 0.99)] + [round(float(x.max()), 1)]  # noqa: E731
        key = os.path.basename(os.path.dirname(path))
        outs[key] = {"kernel_us": round(us, 1), "span_us": round(float(ew.max()), 1),
                     "dur_mean_us": round(float(dur.mean()), 2), "dur_nonempty_mean_us": round(float(dur[ne].mean()), 2),
                     "dur_p50_p90_p99_max": q(dur), "start_p50_p90_max": q(sw)[:2] + [round(float(sw.max()), 1)],
                     "marched": int(c0.sum())}
        first = outs.get("_ref")
        if first is None:
            outs["_ref"] = (c0, s0, d0)
        else:
            c_r, s_r, d_r = first
            same = torch.equal(c0, c_r)
            if same:  # slots bit-exact up to each ray's count
                mask = (torch.arange(tr.max_samples, device=dev)[None, :] < c0[:, None]).flatten()
                same = torch.equal(s0[mask], s_r[mask]) and torch.equal(d0[mask], d_r[mask])
            outs[key]["bit_exact_vs_first"] = bool(same)
        print(key, json.dumps(outs[key]), flush=True)


if __name__ == "__main__":
    main()
