"""datasets/nerf.py:13-100 of the reference: NeRF-synthetic (Blender) scenes,
transforms_{split}.json + PNGs; poses to [right down front] scaled so the
camera centre lies at radius 1.5 (per-scene radius for Jrender_Dataset)."""
import json
import os

import numpy as np
import torch

from .base import BaseDataset
from .color_utils import read_image
from .ray_utils import get_ray_directions

_JRENDER_RADIUS = {'Easyship': 1.2, 'Scar': 1.8, 'Coffee': 2.5, 'Car': 0.8}
_JRENDER_SHIFT = {'Coffee': (1, 0.4465), 'Car': (0, 0.7)}


class NeRFDataset(BaseDataset):
    def __init__(self, root_dir, split='train', downsample=1.0, **kwargs):
        super().__init__(root_dir, split, downsample)
        self.read_intrinsics()
        if kwargs.get('read_meta', True):
            self.read_meta(split)

    def read_intrinsics(self):
        with open(os.path.join(self.root_dir, "transforms_train.json"), 'r') as f:
            meta = json.load(f)
        w = h = int(800 * self.downsample)
        fx = fy = 0.5 * 800 / np.tan(0.5 * meta['camera_angle_x']) * self.downsample
        K = np.float32([[fx, 0, w / 2], [0, fy, h / 2], [0, 0, 1]])
        self.K = torch.FloatTensor(K)
        self.directions = get_ray_directions(h, w, self.K)
        self.img_wh = (w, h)

    def read_meta(self, split):
        self.rays, self.poses = [], []
        names = ["train", "val"] if split == 'trainval' else [split]
        frames = []
        for nm in names:
            with open(os.path.join(self.root_dir, f"transforms_{nm}.json"), 'r') as f:
                frames += json.load(f)["frames"]
        jrender = 'Jrender_Dataset' in self.root_dir
        folder = self.root_dir.split('/')
        scene = folder[-1] if folder[-1] != '' else folder[-2]
        scale = 1.0
        for frame in frames:
            c2w = np.array(frame['transform_matrix'])[:3, :4]
            if jrender:
                c2w[:, :2] *= -1  # [left up front] to [right down front]
                radius = _JRENDER_RADIUS.get(scene, 1.5)
            else:
                c2w[:, 1:3] *= -1  # [right up back] to [right down front]
                radius = 1.5
            scale = np.linalg.norm(c2w[:, 3]) / radius
            c2w[:, 3] /= scale
            if jrender and scene in _JRENDER_SHIFT:
                ax, sh = _JRENDER_SHIFT[scene]
                c2w[ax, 3] -= sh
            self.poses += [c2w]
            img_path = os.path.join(self.root_dir, f"{frame['file_path']}.png")
            if os.path.exists(img_path):  # the reference skips unreadable images (try/except)
                self.rays += [read_image(img_path, self.img_wh)]
        self.blender_trans = np.eye(4)
        self.blender_scale = scale
        if jrender and scene in _JRENDER_SHIFT:
            ax, sh = _JRENDER_SHIFT[scene]
            self.blender_trans[ax, 3] += sh
        if len(self.rays) > 0:
            self.rays = torch.FloatTensor(np.stack(self.rays))  # (N_images, hw, 3)
        self.poses = torch.FloatTensor(np.stack(self.poses))  # (N_images, 3, 4)
