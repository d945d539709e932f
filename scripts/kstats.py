#!/usr/bin/env python3
"""Per-kernel statistics of the TIMED region of a bench.py run under
`rocprofv3 --kernel-trace`: bench.py runs --pretrain + --warmup untimed steps
first, so rocprofv3's own --stats averages are dominated by early training
(denser occupancy grid, more samples).  This keeps the dispatches after the
last `--steps` launches of the per-step anchor kernel (adam_kernel: exactly
one per step) and reports count / mean / min / max per kernel, plus the
wall time of that window and the per-stream busy time.

usage: kstats.py run_kernel_trace.csv STEPS [out.csv]
"""
import csv
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    for pre in ("void ", "_ZN3ngp"):
        n = n.replace(pre, "")
    return n[:80]


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    anchors = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    first = anchors[-steps - 1] + 1 if len(anchors) > steps else 0
    win = rows[first:anchors[-1] + 1]
    t0 = int(win[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in win)
    per = defaultdict(list)
    for r in win:
        per[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = sum(sum(v) for v in per.values())
    out = []
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        out.append({"kernel": short(k), "calls": len(v), "calls_per_step": round(len(v) / steps, 3),
                    "avg_us": round(sum(v) / len(v), 2), "min_us": round(min(v), 2), "max_us": round(max(v), 2),
                    "us_per_step": round(sum(v) / steps, 2), "pct": round(100 * sum(v) / tot, 2)})
    print(f"window: {steps} steps, {(t1 - t0) / 1e3 / steps:.1f} us/step wall, "
          f"{tot / steps:.1f} us/step summed kernel time")
    for o in out[:30]:
        print(f"{o['kernel']:80s} {o['calls_per_step']:6.2f}/step {o['avg_us']:9.2f}us avg "
              f"[{o['min_us']:.1f}, {o['max_us']:.1f}] {o['us_per_step']:8.2f}us/step {o['pct']:5.1f}%")
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0]))
            w.writeheader()
            w.writerows(out)


if __name__ == "__main__":
    main()
