"""Probe the ngp_timing_set hook: eager, torch graph capture, raw HIP capture."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "ar-nerf_amd")]
import ctypes
import torch
import vren
import ktimer as KT
L = vren.lib()
H = KT.hip()
n = 1 << 20
p = [torch.zeros(n, device="cuda") for _ in range(4)]
p16 = torch.zeros(n, dtype=torch.float16, device="cuda")
args = lambda: [ctypes.c_void_p(t.data_ptr()) for t in p] + [ctypes.c_void_p(p16.data_ptr())]


def adam():
    vren._ok(L.ngp_adam_step(*args(), n, 1e-2, 0.9, 0.999, 1e-15, 1, 1.0, 1, vren._stream()), "adam")


def counts_err():
    cc = (ctypes.c_int32 * len(KT.NAMES))()
    return L.ngp_timing_counts(cc, len(KT.NAMES)), cc[KT.NAMES.index("adam")]


tm = KT.KernelTimer(slots=1)
for mode in ("global", "thread_local", "relaxed"):
    g = torch.cuda.CUDAGraph()
    tm.arm(0)
    try:
        with torch.cuda.graph(g, capture_error_mode=mode):
            if mode != "global":
                p[3].add_(1.0)  # a node before the first event record
            adam()
        st = "ok"
    except Exception as e:
        st = repr(e)[:200]
    print("torch", mode, "capture:", st, "record err / count", counts_err(), flush=True)
    L.ngp_timing_set(None, 0, 0, 0)
H.hipStreamBeginCapture.argtypes = [ctypes.c_void_p, ctypes.c_int]
H.hipStreamEndCapture.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]
for mode in (0, 1, 2):
    s = torch.cuda.Stream()
    tm.arm(0)
    r0 = H.hipStreamBeginCapture(ctypes.c_void_p(s.cuda_stream), mode)
    with torch.cuda.stream(s):
        try:
            if mode:
                p[3].add_(1.0)
            adam(); st = "ok"
        except Exception as e:
            st = repr(e)[:200]
    gr = ctypes.c_void_p()
    r1 = H.hipStreamEndCapture(ctypes.c_void_p(s.cuda_stream), ctypes.byref(gr))
    print("raw mode", mode, "begin", r0, "launch", st, "end", r1, "record err / count", counts_err(), flush=True)
    L.ngp_timing_set(None, 0, 0, 0)
