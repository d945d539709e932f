#!/usr/bin/env python3
"""The API compositing kernels (ngp_composite_train_fw / _bw) of two library
builds on the same inputs (diagnostic A/B: e.g. the per-lane serial kernels
against the wave-per-ray ones): every output compared bit for bit, and each
build's kernel time.  usage: composite_libs.py LIB_A.so LIB_B.so"""
import ctypes
import json
import os
import sys

import torch

vp = ctypes.c_void_p


def declare(L):
    L.ngp_composite_train_fw.argtypes = [vp, vp, vp, vp, vp, ctypes.c_int64, ctypes.c_float, vp, vp, vp, vp, vp, vp]
    L.ngp_composite_train_bw.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, ctypes.c_int64, vp, vp, vp,
                                         ctypes.c_float, vp, vp, vp]
    L.ngp_composite_train_fw.restype = L.ngp_composite_train_bw.restype = ctypes.c_int
    return L


def main():
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(3)
    R = 8192
    counts = torch.randint(0, 300, (R,), generator=g)
    counts[::7] = 0
    counts[::11] = torch.randint(300, 1024, (counts[::11].numel(),), generator=g)
    starts = torch.cumsum(counts, 0) - counts
    rays_a = torch.stack([torch.arange(R), starts, counts], 1).to(dev)
    N = int(counts.sum())
    sig = (torch.rand(N, generator=g) * 30).to(dev)
    rgbs = torch.rand(N, 3, generator=g).to(dev)
    deltas = (torch.rand(N, generator=g) * 0.01).to(dev)
    ts = torch.cumsum(deltas, 0)
    gop, gdep = torch.randn(R, generator=g).to(dev), torch.randn(R, generator=g).to(dev)
    grgb, gws = torch.randn(R, 3, generator=g).to(dev), torch.randn(N, generator=g).to(dev)
    p = lambda t: vp(t.data_ptr())  # noqa: E731
    res, outs = {}, []
    for path in sys.argv[1:3]:
        L = declare(ctypes.CDLL(os.path.abspath(path)))
        tot = torch.empty(R, dtype=torch.int64, device=dev)
        op, dep, rgb = torch.empty(R, device=dev), torch.empty(R, device=dev), torch.empty(R, 3, device=dev)
        ws = torch.empty(N, device=dev)
        dsig, drgb = torch.empty(N, device=dev), torch.empty(N, 3, device=dev)
        s = vp(torch.cuda.current_stream().cuda_stream)

        def fw():
            assert L.ngp_composite_train_fw(p(sig), p(rgbs), p(deltas), p(ts), p(rays_a), R, 1e-4, p(tot), p(op),
                                            p(dep), p(rgb), p(ws), s) == 0

        def bw():
            assert L.ngp_composite_train_bw(p(gop), p(gdep), p(grgb), p(gws), p(sig), p(rgbs), p(ws), p(deltas),
                                            p(ts), p(rays_a), R, p(op), p(dep), p(rgb), 1e-4, p(dsig), p(drgb),
                                            s) == 0
        fw()
        bw()
        torch.cuda.synchronize()
        times = {}
        for name, f in (("fw_us", fw), ("bw_us", bw)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                f()
            e1.record()
            torch.cuda.synchronize()
            times[name] = round(e0.elapsed_time(e1) * 1e3 / 20, 1)
        res[os.path.basename(os.path.dirname(path))] = times
        outs.append([t.clone() for t in (tot, op, dep, rgb, ws, dsig, drgb)])
    res["bit_identical"] = [bool(torch.equal(a, b)) for a, b in zip(*outs)]
    res["samples"] = N
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
