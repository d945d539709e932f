#!/usr/bin/env python3
"""Host-side cost of replaying a captured HIP graph vs its kernel count and
stream count (diagnostic): graphs of n tiny kernels on 1 or 2 streams,
replayed 200 times; prints host us per replay and GPU us per replay."""
import json
import time

import torch


def bench(n, streams):
    x = torch.zeros(1024, device="cuda")
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        cs = torch.cuda.current_stream()
        for i in range(n):
            if streams == 2 and i % 2:
                side.wait_stream(cs)
                with torch.cuda.stream(side):
                    x.add_(1.0)
                cs.wait_stream(side)
            else:
                x.add_(1.0)
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        g.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return round((t1 - t0) / 200 * 1e6, 1), round((t2 - t0) / 200 * 1e6, 1)


out = {}
for n in (1, 10, 40, 80):
    for st in (1, 2):
        out[f"n{n}_s{st}"] = bench(n, st)
print(json.dumps(out))
