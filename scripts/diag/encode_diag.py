#!/usr/bin/env python3
"""What bounds the forward hash encode (diagnostic; scripts/diag/encode_diag.hip):
on the marched samples of a steady-state Lego-shaped batch (the trainer
pretrained like bench.py), time ngp_hash_encode, the fused encode + MLP
launch, the MLP alone, and the encode variants of encode_diag.hip (level
ranges, XCD-partitioned level sets, dense levels staged in LDS), each
checked bit-exact against ngp_hash_encode.  Prints one JSON line."""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HERE = os.path.join(ROOT, "scripts", "diag")
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd"), HERE]
import torch  # noqa: E402

import hashgrid as HG  # noqa: E402
import synthetic as S  # noqa: E402
import vren  # noqa: E402
from stages import timed  # noqa: E402
from trainer import NGPTrainer  # noqa: E402


def main():
    lib_path = os.path.join(HERE, "libencdiag.so")
    if not os.path.exists(lib_path):
        subprocess.run(["make", "-C", HERE, "libencdiag.so"], check=True)
    D = ctypes.CDLL(lib_path)
    vp = ctypes.c_void_p
    D.ngp_diag_encode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int64, vp, vp, vp, vp, vp,
                                  ctypes.c_int, vp]
    D.ngp_diag_enc_rows.argtypes = [ctypes.c_int, vp, ctypes.c_int64, vp, vp, vp, vp, vp, ctypes.c_int, vp]
    D.ngp_diag_fem.argtypes = [ctypes.c_int, vp, vp, ctypes.c_int64, vp, vp, vp, vp, vp, vp, ctypes.c_int, vp]
    dev = torch.device("cuda")
    scene = S.AnalyticScene(W=800, H=800, n_images=100, scale=0.5)
    gt = scene.gt_images(device=dev)
    dirs, poses = scene.directions.to(dev), scene.poses.to(dev)
    tr = NGPTrainer(scale=0.5, batch_size=8192, device=dev)
    tr.mark_invisible_cells(scene.K, scene.poses, (scene.W, scene.H))
    for _ in range(int(os.environ.get("PRETRAIN", "2000"))):
        tr.train_step(gt, dirs, poses)
    tr.drain()
    torch.cuda.synchronize()
    p, HGL = HG._ptr, HG._lib()

    class _S:  # the current stream at each call (timed() captures on a side stream)
        _as_parameter_ = None

        @property
        def _as_parameter_(self):
            return vren._stream()
    s = _S()
    g = HG.ctypes.byref(tr.grid.desc)
    table = tr.params16[HG.MLP_PARAMS:]
    n_all = int(tr.n_samples.item())
    out = {"n_marched": n_all}
    ctr = torch.zeros(128, dtype=torch.int32, device=dev)
    for tag, n in (("all", n_all), ("155k", min(n_all, 155000))):
        x = tr.xyzs[:n].contiguous()
        d = tr.dirs[:n].contiguous()
        ref = torch.zeros(8, n, 4, dtype=torch.float16, device=dev)
        enc = torch.zeros_like(ref)
        sig, rgb = torch.empty(n, device=dev), torch.empty(n, 3, device=dev)
        st = {"n": n}
        st["hash_encode"] = timed(lambda: vren._ok(HGL.ngp_hash_encode(p(x), n, None, None, g, p(table), p(ref), s),
                                                   "he"))
        st["fused_encode_mlp"] = timed(lambda: vren._ok(HGL.ngp_field_encode_mlp(
            p(x), p(d), n, None, None, g, p(table), p(tr.params16), p(enc), p(sig), p(rgb), None, s), "fem"))
        st["mlp_only"] = timed(lambda: vren._ok(HGL.ngp_field_mlp_forward(
            p(ref), p(d), n, None, None, p(tr.params16), p(sig), p(rgb), None, s), "mf"))
        blocks_lane = max(1, (n + 255) // 256)

        def run(mode, a, b, blocks):
            vren._ok(D.ngp_diag_encode(mode, a, b, p(x), n, None, g, p(table), p(enc), p(ctr), blocks, s), "diag")

        for name, (p0, p1) in {"dense_levels_0_5": (0, 3), "hashed_levels_6_15": (3, 8), "levels_0_3": (0, 2),
                               "all_levels": (0, 8)}.items():
            st[f"range_{name}"] = timed(lambda: run(1, p0, p1, blocks_lane))
        checks = {}
        for name, mode, a, blocks in (("xcd_pairs", 2, 0, 2048), ("xcd_dense_hashed", 3, 0, 2048),
                                      ("lds_levels_2", 4, 2, 256), ("lds_levels_3", 4, 3, 256)):
            enc.zero_()
            st[name] = timed(lambda: run(mode, a, 0, blocks))
            torch.cuda.synchronize()
            checks[name] = bool(torch.equal(enc.view(torch.int16), ref.view(torch.int16)))
        # the pipelined fused forward (waves per block, blocks) vs ngp_field_encode_mlp, bit for bit
        sig_r, rgb_r, enc_r = sig.clone(), rgb.clone(), torch.zeros_like(ref)
        vren._ok(HGL.ngp_field_encode_mlp(p(x), p(d), n, None, None, g, p(table), p(tr.params16), p(enc_r), p(sig_r),
                                          p(rgb_r), None, s), "fem_ref")
        for nw, blocks in ((8, 256),):
            sig.zero_(); rgb.zero_(); enc.zero_()
            st[f"pipe_w{nw}_b{blocks}"] = timed(lambda: vren._ok(D.ngp_diag_fem(
                nw, p(x), p(d), n, g, p(table), p(tr.params16), p(enc), p(sig), p(rgb), blocks, s), "pipe"))
            torch.cuda.synchronize()
            checks[f"pipe_w{nw}_b{blocks}"] = bool(torch.equal(sig, sig_r) and torch.equal(rgb, rgb_r) and
                                                   torch.equal(enc.view(torch.int16), enc_r.view(torch.int16)))
        # row orders: ray order (identity), samples sorted by the Morton code of their
        # cell at 64^3 / 256^3, a random permutation; grids: the product's / XCD ranges
        G = 64
        xi = ((x - tr.grid.desc.xyz_min[0]) / (2 * 0.5) * G).clamp(0, G - 1).long()
        def morton(c):
            k = torch.zeros(c.shape[0], dtype=torch.int64, device=dev)
            for bit in range(10):
                for d in range(3):
                    k |= ((c[:, d] >> bit) & 1) << (3 * bit + d)
            return k
        orders = {"ray": torch.arange(n, device=dev, dtype=torch.int32),
                  "morton64": torch.argsort(morton(xi)).int(),
                  "morton256": torch.argsort(morton(((x + 0.5) * 256).clamp(0, 255).long())).int(),
                  "random": torch.randperm(n, device=dev).int()}
        for oname, perm in orders.items():
            for mode, blocks in ((0, blocks_lane), (1, 2048), (1, 4096)):
                enc.zero_()
                key = f"rows_{oname}_{'grid' if mode == 0 else 'xcd'}_{blocks}"
                st[key] = timed(lambda: vren._ok(D.ngp_diag_enc_rows(mode, p(x), n, p(perm), g, p(table), p(enc),
                                                                     p(ctr), blocks, s), "rows"))
                torch.cuda.synchronize()
                checks[key] = bool(torch.equal(enc.view(torch.int16), ref.view(torch.int16)))
        st["bit_exact"] = checks
        out[tag] = st
    print(json.dumps(out))


if __name__ == "__main__":
    main()
