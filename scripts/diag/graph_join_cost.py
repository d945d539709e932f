"""Cost of cross-stream dependencies inside a replayed HIP graph (diagnostic).

Each variant is a captured graph of short kernels on the capture stream (a
`torch.cuda._sleep` of S cycles each) with a side branch forked and joined at
different points; the replay wall time per graph (events around 200 replays)
minus the plain chain's tells what a fork / join costs on the critical path:
  chain      : 12 kernels on one stream
  join_early : + a 1-kernel side branch forked after kernel 1, joined before kernel 10
               (its signal is long satisfied when the main stream reaches the join)
  join_late  : + a long side branch (4 sleeps) forked after kernel 1, joined before
               kernel 4 (the main stream waits for it)
  fork_only  : + a side branch forked after kernel 1 and joined only at the end
  two_joins  : join_early's branch + a second branch joined before kernel 6
  join3      : three side branches, all joined before kernel 10
Prints one JSON line."""
import json
import sys

import torch

S = int(sys.argv[1]) if len(sys.argv) > 1 else 20000  # cycles per sleep kernel (~8 us at 2.4 GHz)


def build(kind):
    main = torch.cuda.current_stream()
    sides = [torch.cuda.Stream() for _ in range(3)]
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    cap = torch.cuda.Stream()
    cap.wait_stream(main)
    with torch.cuda.stream(cap):
        with torch.cuda.graph(g, stream=cap):
            cs = torch.cuda.current_stream()
            pending = []
            for k in range(12):
                if k == 1 and kind in ("join_early", "join_late", "fork_only", "two_joins", "join3"):
                    nb = 3 if kind == "join3" else 2 if kind == "two_joins" else 1
                    for b in range(nb):
                        sides[b].wait_stream(cs)
                        with torch.cuda.stream(sides[b]):
                            for _ in range(4 if kind == "join_late" else 1):
                                torch.cuda._sleep(S)
                        pending.append(sides[b])
                join_at = {"join_early": {10: [0]}, "join_late": {4: [0]}, "two_joins": {10: [0], 6: [1]},
                           "join3": {10: [0, 1, 2]}}.get(kind, {})
                for b in join_at.get(k, []):
                    cs.wait_stream(sides[b])
                    pending = [p for p in pending if p is not sides[b]]
                torch.cuda._sleep(S)
            for p in pending:
                cs.wait_stream(p)
    return g


def time_graph(g, reps=200):
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us per replay


out = {"sleep_cycles": S}
for kind in ("chain", "join_early", "join_late", "fork_only", "two_joins", "join3"):
    g = build(kind)
    out[kind + "_us"] = round(min(time_graph(g) for _ in range(3)), 2)
print(json.dumps(out))
