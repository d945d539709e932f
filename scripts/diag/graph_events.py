"""Probe: can HIP timing events be recorded inside a captured graph (torch
external events) and timed after replay on ROCm?"""
import torch

dev = torch.device("cuda", 0)
a = torch.randn(4096, 4096, device=dev)
b = torch.randn(4096, 4096, device=dev)
s = torch.cuda.Stream()
e0 = torch.cuda.Event(enable_timing=True, external=True)
e1 = torch.cuda.Event(enable_timing=True, external=True)
g = torch.cuda.CUDAGraph()
torch.cuda.synchronize()
with torch.cuda.graph(g):
    c = a * 1.0001
    e0.record()
    for _ in range(4):
        c = torch.sin(c) * b
    e1.record()
    d = c + b
for i in range(3):
    g.replay()
    torch.cuda.synchronize()
    print("replay", i, "elapsed ms between external events:", e0.elapsed_time(e1))
# eager reference
x0 = torch.cuda.Event(enable_timing=True); x1 = torch.cuda.Event(enable_timing=True)
x0.record()
for _ in range(4):
    c = torch.sin(c) * b
x1.record(); torch.cuda.synchronize()
print("eager 4 matmuls ms:", x0.elapsed_time(x1))
