"""COLMAP sparse-model readers (the binary format of cameras.bin / images.bin /
points3D.bin, as datasets/colmap_utils.py of the reference reads them),
restated from COLMAP's documented layout (little endian):
  cameras.bin   u64 n; n x {i32 id, i32 model, u64 width, u64 height, f64 params[k(model)]}
  images.bin    u64 n; n x {i32 id, f64 qvec[4] (w,x,y,z), f64 tvec[3], i32 camera_id,
                            name (NUL-terminated), u64 n2d, n2d x {f64 x, f64 y, i64 point3D_id}}
  points3D.bin  u64 n; n x {u64 id, f64 xyz[3], u8 rgb[3], f64 error, u64 len, len x {i32, i32}}"""
import struct
from collections import namedtuple

import numpy as np

Camera = namedtuple("Camera", ["id", "model", "width", "height", "params"])
Point3D = namedtuple("Point3D", ["id", "xyz", "rgb", "error", "image_ids", "point2D_idxs"])

# model id -> (name, number of params)
CAMERA_MODELS = {0: ("SIMPLE_PINHOLE", 3), 1: ("PINHOLE", 4), 2: ("SIMPLE_RADIAL", 4), 3: ("RADIAL", 5),
                 4: ("OPENCV", 8), 5: ("OPENCV_FISHEYE", 8), 6: ("FULL_OPENCV", 12), 7: ("FOV", 5),
                 8: ("SIMPLE_RADIAL_FISHEYE", 4), 9: ("RADIAL_FISHEYE", 5), 10: ("THIN_PRISM_FISHEYE", 12)}


def qvec2rotmat(qvec):
    w, x, y, z = qvec
    return np.array([[1 - 2 * y * y - 2 * z * z, 2 * x * y - 2 * w * z, 2 * z * x + 2 * w * y],
                     [2 * x * y + 2 * w * z, 1 - 2 * x * x - 2 * z * z, 2 * y * z - 2 * w * x],
                     [2 * z * x - 2 * w * y, 2 * y * z + 2 * w * x, 1 - 2 * x * x - 2 * y * y]])


class Image(namedtuple("Image", ["id", "qvec", "tvec", "camera_id", "name", "xys", "point3D_ids"])):
    def qvec2rotmat(self):
        return qvec2rotmat(self.qvec)


def _read(f, fmt):
    fmt = "<" + fmt
    return struct.unpack(fmt, f.read(struct.calcsize(fmt)))


def read_cameras_binary(path):
    cams = {}
    with open(path, "rb") as f:
        (n,) = _read(f, "Q")
        for _ in range(n):
            cid, mid, w, h = _read(f, "iiQQ")
            name, k = CAMERA_MODELS[mid]
            cams[cid] = Camera(cid, name, w, h, np.array(_read(f, "d" * k)))
    return cams


def read_images_binary(path):
    ims = {}
    with open(path, "rb") as f:
        (n,) = _read(f, "Q")
        for _ in range(n):
            v = _read(f, "idddddddi")
            iid, qvec, tvec, cam = v[0], np.array(v[1:5]), np.array(v[5:8]), v[8]
            name = b""
            c = f.read(1)
            while c != b"\x00":
                name += c
                c = f.read(1)
            (n2d,) = _read(f, "Q")
            pts = np.array(_read(f, "ddq" * n2d)).reshape(-1, 3) if n2d else np.zeros((0, 3))
            ims[iid] = Image(iid, qvec, tvec, cam, name.decode(), pts[:, :2], pts[:, 2].astype(np.int64))
    return ims


def read_points3d_binary(path):
    pts = {}
    with open(path, "rb") as f:
        (n,) = _read(f, "Q")
        for _ in range(n):
            v = _read(f, "QdddBBBd")
            (tl,) = _read(f, "Q")
            tr = np.array(_read(f, "ii" * tl)).reshape(-1, 2) if tl else np.zeros((0, 2), np.int64)
            pts[v[0]] = Point3D(v[0], np.array(v[1:4]), np.array(v[4:7]), v[7], tr[:, 0], tr[:, 1])
    return pts


def write_model_binary(root, cameras, images, points):
    """Writer for the same layout (tests and tools)."""
    inv = {v[0]: k for k, v in CAMERA_MODELS.items()}
    with open(f"{root}/cameras.bin", "wb") as f:
        f.write(struct.pack("<Q", len(cameras)))
        for c in cameras.values():
            f.write(struct.pack("<iiQQ", c.id, inv[c.model], c.width, c.height))
            f.write(struct.pack("<" + "d" * len(c.params), *c.params))
    with open(f"{root}/images.bin", "wb") as f:
        f.write(struct.pack("<Q", len(images)))
        for im in images.values():
            f.write(struct.pack("<idddddddi", im.id, *im.qvec, *im.tvec, im.camera_id))
            f.write(im.name.encode() + b"\x00")
            f.write(struct.pack("<Q", 0))
    with open(f"{root}/points3D.bin", "wb") as f:
        f.write(struct.pack("<Q", len(points)))
        for p in points.values():
            f.write(struct.pack("<QdddBBBd", p.id, *p.xyz, *[int(c) for c in p.rgb], p.error))
            f.write(struct.pack("<Q", 0))
