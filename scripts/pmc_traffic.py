#!/usr/bin/env python3
"""profiles/pmc_traffic.json from a scripts/pmc_bench.sh run: HBM-side bytes
per launch of the bench's per-kernel breakdown kernels, from the separate
FETCH_SIZE and WRITE_SIZE passes (KB per dispatch, averaged over the last
dispatches), corrected as MI355X_MICROARCH.md "HBM" prescribes: FETCH_SIZE
doubled (gfx950 tallies 128-B read requests at 64 B); WRITE_SIZE as is (exact
for 16-B streaming stores and dword float atomics; a partial 64-B atomic
request is tallied whole).  Other access widths are uncalibrated (noted).
usage: pmc_traffic.py gpurun_out/pmc_TAG [out.json]"""
import json
import os
import sys

NAMES = {"hash_bwd_kernel": "hash_bwd_coarse", "field_bwd_mlp_kernel": "mlp_bwd", "hash_encode_kernel": "hash_encode",
         "field_bwd_mlp_coop_kernel": "mlp_bwd", "field_encode_mlp_kernel": "hash_encode",
         "field_encode_mlp_reg_kernel": "hash_encode", "field_first_chunk_kernel": "hash_encode_first",
         "encode_coarse_first_kernel": "hash_encode_pre",
         "field_rows_block_kernel": "hash_encode_rows",
         "hash_adam_residual_kernel": "adam",
         "adam_kernel": "adam", "field_fwd_kernel": "field_mlp", "hash_write_kernel": "hash_write",
         "hash_accum_kernel": "hash_accum", "hash_count_kernel": "hash_count", "march_slots_wave_kernel": "march",
         "march_compact_kernel": "march_compact", "composite_loss_wave_kernel": "composite_loss"}  # ktimer names


def parse(path):
    out, cur = {}, None
    for line in open(path):
        if not line.startswith(" "):
            cur = line.strip()
            continue
        k, v = line.split()
        out.setdefault(cur, {})[k] = float(v)
    return out


def key(kname):
    for frag, k in NAMES.items():
        if frag in kname:
            return k
    return None


def main():
    d = sys.argv[1]
    dst = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                             "pmc_traffic.json")
    fetch, write = parse(os.path.join(d, "fetch.txt")), parse(os.path.join(d, "write.txt"))
    res = {}
    for kname, c in fetch.items():
        k = key(kname)
        w = write.get(kname, {})
        if k is None or "FETCH_SIZE" not in c or "WRITE_SIZE" not in w:
            continue
        rd, wr = 2 * c["FETCH_SIZE"] * 1024, w["WRITE_SIZE"] * 1024
        row = {"bytes_per_launch": round(rd + wr), "read_bytes": round(rd), "write_bytes": round(wr),
               "FETCH_SIZE_KB": c["FETCH_SIZE"], "WRITE_SIZE_KB": w["WRITE_SIZE"], "rocprof_kernel": kname,
               "dur_us_fetch_pass": c.get("dur_us"), "dur_us_write_pass": w.get("dur_us")}
        if k == "adam" and k in res:  # two launches per step under one timer name (MLP + coarse, residual):
            a = res[k]                # bytes_per_launch = their mean, so x launches/step = their sum
            for f in ("bytes_per_launch", "read_bytes", "write_bytes"):
                a[f] = round((a[f] + row[f]) / 2)
            a["rocprof_kernel"] += " + " + kname
        elif k not in res or "ILb0E" in res[k]["rocprof_kernel"]:
            res[k] = row  # template variants: not the density-only forward of the occupancy update (1 in 16 steps)
    res["_note"] = ("read = 2 x FETCH_SIZE (gfx950 128-B requests tallied at 64 B); write = WRITE_SIZE; gathers of "
                    "4-16 B lanes and partial-line atomics are uncalibrated widths (MI355X_MICROARCH.md HBM); "
                    "source: " + os.path.basename(os.path.normpath(d)))
    with open(dst, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
