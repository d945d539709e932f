#!/usr/bin/env python3
"""field_fwd launch time vs spatial spread of the samples (diagnostic):
samples uniform in the box (hash-table gathers spread over the whole 23 MB
table, mostly Infinity-Cache served) vs confined to a small cube (the
gathered entries fit the XCD L2s).  Separates gather-memory cost from the
kernel's arithmetic."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd")]
import torch  # noqa: E402

import hashgrid as HG  # noqa: E402

vp = ctypes.c_void_p


def main():
    dev = torch.device("cuda")
    grid = HG.HashGrid(scale=0.5)
    params = HG.init_params(grid, seed=1, device=dev)
    p16 = params.half()
    N = 584_000
    g = torch.Generator(device=dev).manual_seed(0)
    d = torch.nn.functional.normalize(torch.randn(N, 3, device=dev, generator=g), dim=1).contiguous()
    sig, rgb = torch.empty(N, device=dev), torch.empty(N, 3, device=dev)
    enc = torch.empty(N, 32, dtype=torch.float16, device=dev)
    L = HG._lib()
    s = vp(torch.cuda.current_stream().cuda_stream)
    p = lambda t: vp(t.data_ptr())  # noqa: E731
    out = {}
    for name, half_extent in (("box", 0.5), ("cube_0.1", 0.05), ("cube_0.01", 0.005), ("point", 0.0)):
        xyz = ((torch.rand(N, 3, device=dev, generator=g) * 2 - 1) * half_extent).contiguous()
        enc_pm = torch.empty(8, N, 4, dtype=torch.float16, device=dev)
        fe = lambda: L.ngp_hash_encode(p(xyz), N, None, None, ctypes.byref(grid.desc), p(p16[HG.MLP_PARAMS:]),  # noqa
                                       p(enc_pm), s)
        fm = lambda: L.ngp_field_mlp_forward(p(enc_pm), p(d), N, None, None, p(p16), p(sig), p(rgb), None, s)  # noqa
        for nm, f in (("encode", fe), ("mlp", fm)):
            for _ in range(3):
                f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                f()
            e1.record()
            torch.cuda.synchronize()
            out[name + "_" + nm + "_us"] = round(e0.elapsed_time(e1) / 20 * 1e3, 1)
        fn = lambda: L.ngp_field_forward(p(xyz), p(d), N, None, ctypes.byref(grid.desc), p(p16[HG.MLP_PARAMS:]),  # noqa
                                         p(p16), p(sig), p(rgb), p(enc), None, s)
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name + "_us"] = round(e0.elapsed_time(e1) / 20 * 1e3, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
