#!/usr/bin/env python3
"""Split hash-grid backward time (diagnostic; needs a GPU and libdiag.so).

Trains the bench workload for --pretrain steps so samples are in the steady
state, then re-launches the backward on the LAST step's inputs in several
variants: 0 product, 1 no atomics, 2 plain stores, 3 atomics without the
in-wave run merge; over level ranges and persistent-grid caps."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd")]
import torch  # noqa: E402

import hashgrid as HG  # noqa: E402
import synthetic as S  # noqa: E402
from trainer import NGPTrainer  # noqa: E402

D = ctypes.CDLL(os.path.join(ROOT, "scripts", "diag", "libdiag.so"))
vp = ctypes.c_void_p
D.ngp_diag_hash_bwd.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int64, vp, vp,
                                vp, vp, vp, vp]


def main():
    dev = torch.device("cuda")
    sc = S.AnalyticScene(W=800, H=800, n_images=100, scale=0.5)
    gt = sc.gt_images(device=dev)
    dirs, poses = sc.directions.to(dev).contiguous(), sc.poses.to(dev).contiguous()
    tr = NGPTrainer(scale=0.5, batch_size=8192, device=dev, hash_backward="atomic")
    tr.mark_invisible_cells(sc.K, sc.poses, (sc.W, sc.H))
    g = torch.Generator(device=dev).manual_seed(1)
    for _ in range(int(os.environ.get("PRETRAIN", "2000"))):
        img = torch.randint(0, 100, (8192,), device=dev, generator=g)
        pix = torch.randint(0, 800 * 800, (8192,), device=dev, generator=g)
        tr.step(img, pix, gt[img, pix].float() / 255, dirs, poses)
    torch.cuda.synchronize()
    n_act = int(tr.n_active_total.item())
    grad = torch.zeros_like(tr.grad[HG.MLP_PARAMS:])
    s = torch.cuda.current_stream()
    p = lambda t: vp(t.data_ptr())  # noqa: E731

    def run(mode, lo, hi, cap, reps=50):
        def launch():
            st = D.ngp_diag_hash_bwd(mode, lo, hi, cap, p(tr.xyzs), tr.cap, p(tr.n_active_total), p(tr.sample_idx),
                                     ctypes.byref(tr.grid.desc), p(tr.denc), p(grad), vp(s.cuda_stream))
            assert st == 0, st
        for _ in range(3):
            launch()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            launch()
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / reps * 1e3, 1)  # us

    out = {"n_active": n_act, "n_samples": int(tr.n_samples.item())}
    L = HG._lib()
    cap = 8192 * 128
    ws = torch.empty((L.ngp_hash_backward_binned_workspace(cap) + 255) // 256, 64, dtype=torch.int32, device=dev)
    side = torch.cuda.Stream()
    desc = ctypes.byref(tr.grid.desc)
    args = lambda: (p(tr.xyzs), tr.cap, p(tr.n_active_total), p(tr.sample_idx), desc, p(tr.denc))  # noqa: E731

    def atomic(lo, hi, stream):
        assert L.ngp_hash_backward_levels(*args(), p(grad), lo, hi, vp(stream.cuda_stream)) == 0

    def binned(lo, stream):
        assert L.ngp_hash_backward_binned(*args(), p(grad), p(ws), cap, lo, 0, vp(stream.cuda_stream)) == 0

    def timed(fn, reps=30):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / reps * 1e3, 1)

    def hybrid(lo, concurrent):
        def fn():
            if concurrent:
                side.wait_stream(s)
                binned(lo, side)
                atomic(0, lo, s)
                s.wait_stream(side)
            else:
                atomic(0, lo, s)
                binned(lo, s)
        return fn

    out["atomic_all_us"] = timed(lambda: atomic(0, 16, s))
    out["binned_all_us"] = timed(lambda: binned(0, s))
    for lo in (4, 6, 8, 10):
        out[f"hybrid{lo}_seq_us"] = timed(hybrid(lo, False))
        out[f"hybrid{lo}_conc_us"] = timed(hybrid(lo, True))
        out[f"atomic_0-{lo}_us"] = timed(lambda: atomic(0, lo, s))
        out[f"binned_{lo}-16_us"] = timed(lambda: binned(lo, s))
    binned(0, s)
    D.ngp_diag_hash_write.argtypes = [ctypes.c_int, vp, ctypes.c_int64, vp, vp, vp, vp, vp, vp, ctypes.c_int64,
                                      ctypes.c_int, vp]
    for mode in (0, 1, 2, 3, 7):
        out[f"write_mode{mode}_us"] = timed(lambda: D.ngp_diag_hash_write(
            mode, p(tr.xyzs), tr.cap, p(tr.n_active_total), p(tr.sample_idx), desc, p(tr.denc), p(grad), p(ws),
            cap, 0, vp(s.cuda_stream)), reps=20)
    binned(0, s)  # consistent workspace for the accum variants
    D.ngp_diag_hash_accum.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, vp, ctypes.c_int64, ctypes.c_int, vp]
    for mode in (0, 1, 3):
        out[f"accum_mode{mode}_us"] = timed(lambda: D.ngp_diag_hash_accum(mode, 1024, desc, p(grad), p(ws), cap, 0,
                                                                           vp(s.cuda_stream)), reps=20)
    if os.environ.get("BINNED_ONLY"):
        print(json.dumps(out))
        return
    for mode in (0, 1, 2, 3):
        out[f"mode{mode}_all"] = run(mode, 0, 16, 8192)
    for cap in (512, 1024, 2048, 4096):
        out[f"mode0_cap{cap}"] = run(0, 0, 16, cap)
    for lo, hi in ((0, 4), (4, 8), (8, 12), (12, 16)):
        out[f"mode0_l{lo}-{hi}"] = run(0, lo, hi, 8192)
        out[f"mode3_l{lo}-{hi}"] = run(3, lo, hi, 8192)
        out[f"mode2_l{lo}-{hi}"] = run(2, lo, hi, 8192)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
