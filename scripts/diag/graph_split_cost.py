"""How to run a side branch beside a replayed chain of kernels (diagnostic).

A "step" = 12 short kernels on the main stream (torch.cuda._sleep of S cycles)
plus one side kernel that may run beside kernels 2-9 (forked after kernel 1,
joined before kernel 10).  Variants, each timed over 200 steps back to back
(us per step, best of 3):
  chain    : one graph, the 12 main kernels only (no side work at all)
  serial   : one graph, the side kernel inline on the main stream (13 kernels)
  forked   : one graph with the side kernel as a captured fork / join
  split    : three single-stream graphs on the main stream (kernels 0-1, 2-9,
             10-11) and a one-kernel graph on the side stream, ordered by events
             recorded / waited between the replays
  eager    : the same three main graphs, the side kernel launched eagerly on the
             side stream between event waits
Prints one JSON line."""
import json
import sys

import torch

S = int(sys.argv[1]) if len(sys.argv) > 1 else 20000


def capture(fn, stream):
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        with torch.cuda.graph(g, stream=stream):
            fn()
    torch.cuda.synchronize()
    return g


def sleeps(n):
    def f():
        for _ in range(n):
            torch.cuda._sleep(S)
    return f


main = torch.cuda.Stream()
side = torch.cuda.Stream()
cap = torch.cuda.Stream()


def forked_body():
    cs = torch.cuda.current_stream()
    torch.cuda._sleep(S)
    torch.cuda._sleep(S)
    side.wait_stream(cs)
    with torch.cuda.stream(side):
        torch.cuda._sleep(S)
    for _ in range(8):
        torch.cuda._sleep(S)
    cs.wait_stream(side)
    torch.cuda._sleep(S)
    torch.cuda._sleep(S)


g_chain = capture(sleeps(12), cap)
g_serial = capture(sleeps(13), cap)
g_forked = capture(forked_body, cap)
g_a, g_b, g_c = capture(sleeps(2), cap), capture(sleeps(8), cap), capture(sleeps(2), cap)
g_s = capture(sleeps(1), cap)


def step_single(g):
    def f():
        with torch.cuda.stream(main):
            g.replay()
    return f


def step_split(eager):
    def f():
        with torch.cuda.stream(main):
            g_a.replay()
            e1 = torch.cuda.Event()
            e1.record(main)
        side.wait_event(e1)
        with torch.cuda.stream(side):
            if eager:
                torch.cuda._sleep(S)
            else:
                g_s.replay()
            e2 = torch.cuda.Event()
            e2.record(side)
        with torch.cuda.stream(main):
            g_b.replay()
            main.wait_event(e2)
            g_c.replay()
    return f


def timeit(step, reps=200):
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(main)
    for _ in range(reps):
        step()
    b.record(main)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


out = {"sleep_cycles": S}
for name, st in (("chain", step_single(g_chain)), ("serial", step_single(g_serial)),
                 ("forked", step_single(g_forked)), ("split", step_split(False)), ("eager", step_split(True))):
    out[name + "_us"] = round(min(timeit(st) for _ in range(3)), 2)
print(json.dumps(out))
