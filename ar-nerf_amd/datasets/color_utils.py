"""datasets/color_utils.py:11-41 of the reference (PNG path; EXR needs cv2's
OpenEXR reader, out of scope)."""
import numpy as np
import torch
import torch.nn.functional as F

from .png import read_png


def srgb_to_linear(img):
    limit = 0.04045
    return np.where(img > limit, ((img + 0.055) / 1.055) ** 2.4, img / 12.92)


def linear_to_srgb(img):
    limit = 0.0031308
    img = np.where(img > limit, 1.055 * img ** (1 / 2.4) - 0.055, 12.92 * img)
    img[img > 1] = 1  # "clamp" tonemapper
    return img


def _resize(img, wh):
    """cv2.resize(img, (w, h)) with INTER_LINEAR (half-pixel centres, no
    antialiasing) on float32 (H, W, C)."""
    w, h = wh
    if img.shape[1] == w and img.shape[0] == h:
        return img
    t = torch.from_numpy(np.ascontiguousarray(img)).permute(2, 0, 1)[None]
    t = F.interpolate(t, size=(h, w), mode="bilinear", align_corners=False, antialias=False)
    return t[0].permute(1, 2, 0).numpy()


def read_image(img_path, img_wh, blend_a=True, exr_file=False):
    """-> float32 (h*w, 3): RGBA blended onto white (blend_a) or black."""
    if exr_file:
        raise NotImplementedError("EXR images need OpenCV's OpenEXR reader (not available)")
    if img_path.lower().endswith(".png"):
        img = read_png(img_path).astype(np.float32) / 255.0
    else:  # JPEG etc.: Pillow (what imageio itself uses for these formats)
        from PIL import Image
        img = np.asarray(Image.open(img_path)).astype(np.float32) / 255.0
        if img.ndim == 2:
            img = img[..., None].repeat(3, -1)
    if img.shape[2] == 4:  # blend A to RGB
        if blend_a:
            img = img[..., :3] * img[..., -1:] + (1 - img[..., -1:])
        else:
            img = img[..., :3] * img[..., -1:]
    img = _resize(img, img_wh)
    return img.reshape(-1, img.shape[-1])
