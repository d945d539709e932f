#!/usr/bin/env python3
"""LDS atomic throughput (diagnostic): lane-ops per CU-cycle for ds_add_f32 /
u32 / f64 and plain read-modify-write, random and conflict-free addresses."""
import ctypes
import json
import os

import torch

D = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libdiag.so"))
D.ngp_diag_lds_atomics.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
out = torch.zeros(256, device="cuda")
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
res = {}
for kind, name in enumerate(["f32", "u32", "f64", "plain_rmw", "f32_linear"]):
    def run(it):
        assert D.ngp_diag_lds_atomics(kind, it, ctypes.c_void_p(out.data_ptr()), s) == 0
    run(64)
    times = []
    for it in (256, 1280):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); run(it); e1.record(); torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) * 1e-3)
    dt = (times[1] - times[0]) / 1024  # s per iteration (1024 threads x 256 CUs)
    res[name] = {"cycles_per_lane_per_CU": round(dt * 2.4e9 / 1024, 3), "Gops_chip": round(1024 * 256 / dt / 1e9, 1)}
print(json.dumps(res))
