#!/usr/bin/env python3
"""Recompute the bench line's per-op roofline fractions from a rocprofv3
kernel trace of the SAME bench command (VERDICT r04 "Next" #1).

bench.py brackets its roofline window -- the graph replays whose device
probes give the line's `ops` / `roofline` -- with two trace_marker_kernel
launches (ngp_trace_marker).  This script keeps the dispatches between the
markers, averages each op's member kernels' durations (End - Start of the
dispatch) over the window, and recomputes `achieved` / `frac` with the line's
own algorithmic work per step.  It prints, per op, the probe-based figure, the
trace-based figure and their ratio, and writes the window's per-kernel
statistics (the kstats the comparison used).

usage: roofline_check.py run_kernel_trace.csv bench_line.json [kstats_out.txt]
"""
import csv
import json
import sys
from collections import defaultdict

# probe name -> substring of the product kernel's (mangled or demangled) name
KERNEL_OF = {
    "march": "march_slots_wave_kernel",
    "first_chunk": "field_first_chunk_kernel",
    "field_encode_mlp": ("field_encode_mlp_reg_kernel", ("ILb1E", "<true>")),
    "pre_encode": "encode_coarse_first_kernel",
    "composite_loss": "composite_loss_wave_kernel",
    "mlp_bwd": "field_bwd_mlp_coop_kernel",
    "hash_bwd_coarse": ("hash_bwd_", ("hash_bwd_kernel", "hash_bwd_wide_kernel")),
    "hash_count": "hash_count_kernel",
    "hash_write": "hash_write_kernel",
    "hash_accum": "hash_accum_kernel",
    "adam": "adam_kernel",
}


def matches(probe, name):
    k = KERNEL_OF[probe]
    if isinstance(k, tuple):
        return k[0] in name and any(t in name for t in k[1])
    return k in name and "residual" not in name


def main():
    trace, line_path = sys.argv[1], sys.argv[2]
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "trace_marker_kernel" in r["Kernel_Name"]]
    if len(marks) < 2:
        sys.exit("no trace_marker_kernel pair in the trace")
    a, b = marks[-2], marks[-1]
    t_lo, t_hi = int(rows[a]["End_Timestamp"]), int(rows[b]["Start_Timestamp"])
    win = [r for r in rows[a + 1:b] if int(r["Start_Timestamp"]) >= t_lo]
    line = json.loads(open(line_path).read().strip().splitlines()[-1])
    steps = line["roofline"]["units_check"]["steps_run"]["roofline"]  # the probed window's steps
    per = defaultdict(list)
    for r in win:
        per[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = []
    print(f"roofline window: {steps} steps, {(t_hi - t_lo) / 1e3 / steps:.1f} us/step wall between the markers, "
          f"{len(win)} dispatches")
    for op, r in line["ops"].items():
        ms = 0.0
        n = []
        for probe in r["kernels"]:
            ds = [d for k, v in per.items() if matches(probe, k) for d in v]
            if not ds:
                break
            ms += sum(ds) / len(ds) / 1e3
            n.append(len(ds))
        else:
            work = r["work_per_step"]
            ach = work / (ms * 1e-3) / (1e9 if r["unit"] == "GB/s" else 1e12)
            frac = ach / r["peak"]
            out.append((op, r["frac"], frac, r["ms_per_step"], ms, n))
            continue
    for op, r in line["ops"].items():  # per member kernel: probe span vs dispatch duration
        for probe in r["kernels"]:
            ds = [d for k, v in per.items() if matches(probe, k) for d in v]
            pm = r.get("kernel_ms", {}).get(probe)
            if ds and pm:
                td = sum(ds) / len(ds)
                print(f"  {op:16s} {probe:18s} probe {pm * 1e3:8.1f} us | trace {td:8.1f} us | trace - probe "
                      f"{td - pm * 1e3:6.1f} us")
    for op, fp, ft, mp, mt, n in out:
        print(f"{op:16s} probes: {mp * 1e3:8.1f} us/step frac {fp:.4f} | trace: {mt * 1e3:8.1f} us/step frac {ft:.4f} "
              f"(launches {n}) | ratio {ft / fp:.3f}")
    roof = line["roofline"]["op"]
    for op, fp, ft, *_ in out:
        if op == roof:
            print(f"roofline op {roof}: line frac {fp:.4f}, trace frac {ft:.4f}, agree within "
                  f"{abs(ft / fp - 1) * 100:.1f} %")
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            f.write(f"# kernel durations inside the roofline window ({steps} steps between the trace markers)\n")
            tot = sum(sum(v) for v in per.values())
            for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
                nm = k.split("(")[0].replace("void ", "")[:90]
                f.write(f"{nm:90s} calls {len(v):5d} avg_us {sum(v) / len(v):9.2f} us_per_step {sum(v) / steps:9.2f} "
                        f"pct {100 * sum(v) / tot:5.1f}\n")


if __name__ == "__main__":
    main()
