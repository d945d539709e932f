#!/usr/bin/env python3
"""Launch time vs sample count for the field kernels (diagnostic): separates
per-launch fixed cost (weight staging, reductions) from per-sample cost."""
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
    with torch.no_grad():
        p16[HG.MLP_PARAMS:].uniform_(-0.5, 0.5)
    N = 600_000
    g = torch.Generator(device=dev).manual_seed(0)
    xyz = (torch.rand(N, 3, device=dev, generator=g) - 0.5) * 0.8
    d = torch.nn.functional.normalize(torch.randn(N, 3, device=dev, generator=g), dim=1)
    sig, rgb = torch.empty(N, device=dev), torch.empty(N, 3, device=dev)
    enc = torch.empty(N, 32, dtype=torch.float16, device=dev)
    dsig, drgb = torch.randn(N, device=dev, generator=g) * 1e-3, torch.randn(N, 3, device=dev, generator=g) * 1e-3
    denc = torch.empty(N, 32, device=dev)
    grad = torch.zeros(params.numel(), device=dev)
    L = HG._lib()
    s = vp(torch.cuda.current_stream().cuda_stream)
    p = lambda t: vp(t.data_ptr())  # noqa: E731

    def t_of(fn, reps=30):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / reps * 1e3, 1)

    out = {}
    for n in (4096, 16384, 65536, 131072, 262144, 524288):
        fwd = lambda: L.ngp_field_forward(p(xyz), p(d), n, None, ctypes.byref(grid.desc), p(p16[HG.MLP_PARAMS:]),  # noqa
                                          p(p16), p(sig), p(rgb), p(enc), None, s)
        mlp = lambda: L.ngp_field_backward_mlp(p(d), n, None, None, p(enc), 0, p(p16), p(dsig), p(drgb), p(denc),  # noqa
                                               p(grad), s)
        hsh = lambda: L.ngp_hash_backward(p(xyz), n, None, None, ctypes.byref(grid.desc), p(denc),  # noqa
                                          p(grad[HG.MLP_PARAMS:]), s)
        out[n] = {"field_fwd_us": t_of(fwd), "mlp_bwd_us": t_of(mlp), "hash_bwd_us": t_of(hsh)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
