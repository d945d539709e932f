#!/usr/bin/env python3
"""Random gather rate (lane-granular loads) vs width, table size, occupancy."""
import ctypes
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    L = ctypes.CDLL(os.path.join(HERE, "libgather.so"))
    L.diag_gather.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                              ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda")
    out = torch.zeros(1 << 22, device=dev)
    res = {}
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for tb in (2 << 20, 24 << 20):
        table = torch.randint(0, 255, (tb,), dtype=torch.uint8, device=dev)
        for width in (4, 8, 16):
            for blocks in (256 * 2, 256 * 8):
                iters = 64
                f = lambda: L.diag_gather(ctypes.c_void_p(table.data_ptr()), tb, width, blocks, iters, 7,  # noqa
                                          ctypes.c_void_p(out.data_ptr()), s)
                f()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    f()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / 5 * 1e3
                gathers = blocks * 256 * iters * 8
                res[f"T{tb >> 20}MB_W{width}_b{blocks}"] = {"us": round(us, 1), "Ggathers_s": round(gathers / us / 1e3, 1),
                                                           "per_cu_per_clk": round(gathers / 256 / (us * 2400), 3)}
    print(json.dumps(res, indent=0))


if __name__ == "__main__":
    main()
