#!/usr/bin/env python3
"""Average PMC counters per kernel over the last N dispatches of each
(the timed steps of a scripts/pmc_bench.sh run).  usage: pmc_summary.py DIR [N]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10
    res = defaultdict(dict)
    for f in glob.glob(os.path.join(root, "**", "run_counter_collection.csv"), recursive=True):
        per = defaultdict(lambda: defaultdict(dict))
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
            per[name][int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
            per[name][int(r["Dispatch_Id"])]["dur_us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        for name, disp in per.items():
            ids = sorted(disp)[-n:]
            for c in disp[ids[0]]:
                res[name][c] = sum(disp[i].get(c, 0.0) for i in ids) / len(ids)
    for name, cs in sorted(res.items()):
        print(name)
        for c, v in sorted(cs.items()):
            print(f"    {c:36s} {v:16.1f}")


if __name__ == "__main__":
    main()
