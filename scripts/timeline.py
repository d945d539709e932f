#!/usr/bin/env python3
"""One step's kernel timeline (start offset, duration, queue, name) from a
rocprofv3 kernel trace, plus per-queue busy time and the idle gaps between
consecutive kernels of the main queue, over the last STEPS steps.
usage: timeline.py run_kernel_trace.csv STEPS [step_index_from_end] [anchor]
(anchor: a substring of the kernel that ends a step; default adam_kernel -- use e.g.
sample_batch_kernel for the data-parallel step, which runs one Adam launch per bucket)"""
import csv
import sys
from collections import defaultdict


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    back = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    anchor = sys.argv[4] if len(sys.argv) > 4 else "adam_kernel"
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    anch = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    win = rows[anch[-steps - 1] + 1:anch[-1] + 1]
    q = defaultdict(list)
    for r in win:
        q[r["Queue_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    main_q = max(q, key=lambda k: len(q[k]))
    v = sorted(q[main_q])
    gaps = [max(0, v[i + 1][0] - v[i][1]) for i in range(len(v) - 1)]
    t0, t1 = win[0]["Start_Timestamp"], max(int(r["End_Timestamp"]) for r in win)
    print(f"wall/step {(t1 - int(t0)) / 1e3 / steps:.1f} us; main queue {main_q}: {len(v) / steps:.1f} kernels/step, "
          f"idle gaps {sum(gaps) / 1e3 / steps:.1f} us/step (median gap {sorted(gaps)[len(gaps) // 2] / 1e3:.2f} us)")
    for k, vv in q.items():
        vv.sort()
        busy, cs, ce = 0, vv[0][0], vv[0][1]
        for s, e in vv[1:]:
            if s > ce:
                busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        print(f"  queue {k}: {len(vv) / steps:.1f} kernels/step, busy {busy / 1e3 / steps:.1f} us/step")
    # time with no kernel running on any queue (dependency / launch latency)
    allv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in win)
    idle, ce = 0, allv[0][1]
    for st, en in allv[1:]:
        if st > ce:
            idle += st - ce
        ce = max(ce, en)
    print(f"  all queues idle {idle / 1e3 / steps:.1f} us/step")
    seg = rows[anch[-back - 1] + 1:anch[-back] + 1]
    prev_end = int(rows[anch[-back - 1]]["End_Timestamp"])
    print(f"  gap from the previous step's adam end to this step's first kernel: "
          f"{(int(seg[0]['Start_Timestamp']) - prev_end) / 1e3:.1f} us")
    s0 = int(seg[0]["Start_Timestamp"])
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - s0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{r['Queue_Id']} {r['Kernel_Name'][:70]}")


if __name__ == "__main__":
    main()
