"""Minimal PNG decoder (8-bit gray / gray+alpha / RGB / RGBA, non-interlaced)
for the NeRF-synthetic images: the reference reads them with imageio
(datasets/color_utils.py:33), which is not installed here.  zlib inflate +
the five PNG scanline filters, vectorised per row with numpy."""
import struct
import zlib

import numpy as np

_CH = {0: 1, 2: 3, 4: 2, 6: 4}


def _paeth(a, b, c):
    p = a.astype(np.int16) + b - c
    pa, pb, pc = np.abs(p - a), np.abs(p - b), np.abs(p - c)
    return np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, c)).astype(np.uint8)


def read_png(path):
    """-> uint8 array (H, W, C)."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:8] != b"\x89PNG\r\n\x1a\n":
        raise ValueError(f"{path}: not a PNG file")
    pos, idat, hdr = 8, [], None
    while pos < len(data):
        n, kind = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        pos += 12 + n
        if kind == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", body)
        elif kind == b"IDAT":
            idat.append(body)
        elif kind == b"IEND":
            break
    W, H, depth, ctype, _, _, interlace = hdr
    if depth != 8 or ctype not in _CH or interlace:
        raise ValueError(f"{path}: only 8-bit non-interlaced gray/RGB(A) PNGs are supported")
    C = _CH[ctype]
    raw = np.frombuffer(zlib.decompress(b"".join(idat)), np.uint8).reshape(H, 1 + W * C)
    out = np.zeros((H, W * C), np.uint8)
    prev = np.zeros(W * C, np.uint8)
    for y in range(H):
        ft, line = raw[y, 0], raw[y, 1:].copy()
        if ft == 0:
            cur = line
        elif ft == 2:
            cur = (line + prev).astype(np.uint8)
        elif ft in (1, 3, 4):  # depend on the reconstructed left neighbour: per pixel
            cur = np.zeros_like(line)
            for x in range(0, W * C, C):
                a = cur[x - C:x] if x >= C else np.zeros(C, np.uint8)
                b, c = prev[x:x + C], prev[x - C:x] if x >= C else np.zeros(C, np.uint8)
                if ft == 1:
                    pred = a
                elif ft == 3:
                    pred = ((a.astype(np.uint16) + b) >> 1).astype(np.uint8)
                else:
                    pred = _paeth(a, b, c)
                cur[x:x + C] = line[x:x + C] + pred
        else:
            raise ValueError(f"{path}: bad filter type {ft}")
        out[y] = cur
        prev = cur
    return out.reshape(H, W, C)


def write_png(path, img):
    """uint8 (H, W, C) -> PNG (filter 0), for tests and tools."""
    img = np.ascontiguousarray(img, np.uint8)
    H, W, C = img.shape
    ctype = {1: 0, 2: 4, 3: 2, 4: 6}[C]
    raw = b"".join(b"\x00" + img[y].tobytes() for y in range(H))

    def chunk(kind, body):
        return struct.pack(">I", len(body)) + kind + body + struct.pack(">I", zlib.crc32(kind + body) & 0xffffffff)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", W, H, 8, ctype, 0, 0, 0)) +
                chunk(b"IDAT", zlib.compress(raw)) + chunk(b"IEND", b""))
