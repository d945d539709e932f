#!/usr/bin/env python3
"""Per-kernel time of the test-time render frames in a rocprofv3
--kernel-trace CSV of scripts/render_profile.py: the window starts at the
first render_begin_kernel (everything before is training).
usage: render_kstats.py run_kernel_trace.csv FRAMES"""
import csv
import sys
from collections import defaultdict


def main():
    path, frames = sys.argv[1], int(sys.argv[2])
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    first = next(i for i, r in enumerate(rows) if "render_begin" in r["Kernel_Name"])
    win = rows[first:]
    t0, t1 = int(win[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in win)
    per = defaultdict(list)
    for r in win:
        per[r["Kernel_Name"].split("(")[0][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = sum(sum(v) for v in per.values())
    n_begin = len(per.get(next(k for k in per if "render_begin" in k), []))
    print(f"window {(t1 - t0) / 1e3:.0f} us over {n_begin} frame starts; summed kernel time {tot:.0f} us")
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:70s} {len(v) / n_begin:7.1f}/frame {sum(v) / len(v):8.2f} us avg  "
              f"{sum(v) / n_begin:9.1f} us/frame {100 * sum(v) / tot:5.1f}%")
    # per-iteration durations of the last graph-rendered frame
    starts = [i for i, r in enumerate(rows) if "render_begin" in r["Kernel_Name"]]
    last = rows[starts[-1]:]
    seq = defaultdict(list)
    for r in last:
        n = r["Kernel_Name"]
        for key in ("render_march", "hash_encode", "field_fwd_kernelILb1ELb1", "render_composite"):
            if key in n:
                seq[key].append(round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, 1))
        if "render_finish" in n:
            break
    for k, v in seq.items():
        print(f"last frame {k}: {v}")


if __name__ == "__main__":
    main()
