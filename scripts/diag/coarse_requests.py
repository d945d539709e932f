#!/usr/bin/env python3
"""Count the coarse hash backward's memory-side atomic requests (distinct
64-B lines per wave instruction) on real gradient-carrying samples
(scripts/diag/active_dump.py -> active.npz) under different merge schemes:

  wave16   the kernel as built (hash_bwd_kernel: 16 consecutive samples per
           wave, lanes (s, cx, f), one instruction per (level, yz corner),
           runs of equal corners at lane stride 4 merged, heads add)
  blockS   every (level, 64-B line) a block of S consecutive samples touches,
           added once per block (an LDS-privatised block image, flushed per line)
  all      every line touched by the step once (the floor)

usage: coarse_requests.py active.npz [levels_hi=8]"""
import sys

import numpy as np

SCALES = [15.0, 20.112, 26.858, 35.758, 47.503, 63.0, 83.449, 110.43]
RES = [16, 22, 28, 37, 49, 65, 85, 112]
SIZES = [4096, 10648, 21952, 50656, 117656, 274632, 524288, 524288]
OFFS = [0, 4096, 14744, 36696, 87352, 205008, 479640, 1003928]
DENSE = [True] * 6 + [False] * 2


def scale_exact(l):
    b = np.float32(np.exp(np.log(2048 * 0.5 / 16) / 15))
    return np.float32(np.exp2(np.float32(l) * np.log2(b)) * 16 - 1)


def corner_idx(p, l):
    """p (n, 3) uint64 grid coords -> table entry (level-relative)"""
    if DENSE[l]:
        r = RES[l]
        i = p[:, 0] + p[:, 1] * r + p[:, 2] * r * r
        return np.where(i >= SIZES[l], i - SIZES[l], i) % SIZES[l]
    i = (p[:, 0] * 1) ^ ((p[:, 1] * 2654435761) & 0xFFFFFFFF) ^ ((p[:, 2] * 805459861) & 0xFFFFFFFF)
    return (i & 0xFFFFFFFF) % SIZES[l]


def level_corners(xyz, l):
    x = (xyz + 0.5).astype(np.float32)  # (x - min) / (max - min) with min -0.5, max 0.5
    p = np.float32(SCALES[l]) * x + np.float32(0.5)
    fl = np.floor(p)
    pg = fl.astype(np.int64).astype(np.uint64)
    out = np.empty((xyz.shape[0], 8), dtype=np.int64)
    for c in range(8):
        d = np.array([c & 1, (c >> 1) & 1, (c >> 2) & 1], dtype=np.uint64)
        out[:, c] = corner_idx(pg + d, l).astype(np.int64)
    return out  # corner c = cx | cy << 1 | cz << 2


def wave16(cor):
    """requests of the kernel as built for one level: cor (n, 8)"""
    n = cor.shape[0]
    nw = (n + 15) // 16
    pad = nw * 16 - n
    c = np.concatenate([cor, np.full((pad, 8), -1, np.int64)]).reshape(nw, 16, 8)
    total = 0
    for yz in range(4):
        for cx in range(2):
            k = cx | (yz << 1)
            v = c[:, :, k]
            head = np.ones_like(v, dtype=bool)
            head[:, 1:] = v[:, 1:] != v[:, :-1]
            head &= v >= 0
            # f = 0, 1 lanes: floats 2 idx + f -> one 8-B pair, same line
            line = np.where(head, (2 * v) // 16, -1)  # 16 floats per 64-B line
            if cx == 0:
                lines0 = line
            else:
                both = np.concatenate([lines0, line], axis=1)  # one instruction covers cx = 0, 1
                s = np.sort(both, axis=1)
                distinct = (s[:, 1:] != s[:, :-1]) & (s[:, 1:] >= 0)
                total += int(distinct.sum() + (s[:, 0] >= 0).sum())
    return total


def block_lines(cor, S):
    n = cor.shape[0]
    blk = np.repeat(np.arange((n + S - 1) // S), 1)[np.arange(n) // S]
    lines = (2 * cor) // 16
    key = blk[:, None].astype(np.int64) * (1 << 32) + lines
    return len(np.unique(key))


def main():
    d = np.load(sys.argv[1])
    lv_hi = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    for s in range(4):
        k = f"xyz{s}"
        if k not in d:
            continue
        xyz = d[k].astype(np.float32)
        n = xyz.shape[0]
        row = {"wave16": 0, "block256": 0, "block1024": 0, "block4096": 0, "all": 0}
        per_level = []
        for l in range(lv_hi):
            cor = level_corners(xyz, l)
            w = wave16(cor)
            b2 = block_lines(cor, 256)
            b10 = block_lines(cor, 1024)
            b40 = block_lines(cor, 4096)
            a = len(np.unique((2 * cor) // 16))
            row["wave16"] += w
            row["block256"] += b2
            row["block1024"] += b10
            row["block4096"] += b40
            row["all"] += a
            per_level.append((l, w, b2, b10, a))
        print(f"step {s}: {n} active samples; requests per step: " +
              ", ".join(f"{k} {v} ({v / n:.3f}/sample)" for k, v in row.items()))
        for l, w, b2, b10, a in per_level:
            print(f"   level {l}: wave16 {w}  block256 {b2}  block1024 {b10}  all {a}")


if __name__ == "__main__":
    main()
