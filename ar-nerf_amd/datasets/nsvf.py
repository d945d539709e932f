"""datasets/nsvf.py:13-100 of the reference: NSVF-format scenes
(Synthetic_NeRF / Synthetic_NSVF, BlendedMVS, TanksAndTemple): intrinsics.txt,
bbox.txt, rgb/{0,1,2}_*.png, pose/{0,1,2}_*.txt (c2w, [right down front]).
Poses are shifted to the bbox centre and scaled so the scene lies in
[-0.5, 0.5] (scale = 1.05 * half the largest bbox side; x1.2 Mic, x1.1 Lego)."""
import glob
import os

import numpy as np
import torch

from .base import BaseDataset
from .color_utils import read_image
from .ray_utils import get_ray_directions


class NSVFDataset(BaseDataset):
    def __init__(self, root_dir, split='train', downsample=1.0, **kwargs):
        super().__init__(root_dir, split, downsample)
        self.read_intrinsics()
        if kwargs.get('read_meta', True):
            xyz_min, xyz_max = np.loadtxt(os.path.join(root_dir, 'bbox.txt'))[:6].reshape(2, 3)
            self.shift = (xyz_max + xyz_min) / 2
            self.scale = (xyz_max - xyz_min).max() / 2 * 1.05  # enlarge a little
            if 'Mic' in self.root_dir:  # the reference's per-scene bound fixes
                self.scale *= 1.2
            elif 'Lego' in self.root_dir:
                self.scale *= 1.1
            self.read_meta(split)

    def read_intrinsics(self):
        if 'Synthetic' in self.root_dir or 'Ignatius' in self.root_dir:
            with open(os.path.join(self.root_dir, 'intrinsics.txt')) as f:
                fx = fy = float(f.readline().split()[0]) * self.downsample
            if 'Synthetic' in self.root_dir:
                w = h = int(800 * self.downsample)
            else:
                w, h = int(1920 * self.downsample), int(1080 * self.downsample)
            K = np.float32([[fx, 0, w / 2], [0, fy, h / 2], [0, 0, 1]])
        else:
            K = np.loadtxt(os.path.join(self.root_dir, 'intrinsics.txt'), dtype=np.float32)[:3, :3]
            if 'BlendedMVS' in self.root_dir:
                w, h = int(768 * self.downsample), int(576 * self.downsample)
            elif 'Tanks' in self.root_dir:
                w, h = int(1920 * self.downsample), int(1080 * self.downsample)
            else:
                raise ValueError(f"unknown NSVF scene family for {self.root_dir}")
            K[:2] *= self.downsample
        self.K = torch.FloatTensor(K)
        self.directions = get_ray_directions(h, w, self.K)
        self.img_wh = (w, h)

    def _normalise(self, c2w):
        c2w[:, 3] -= self.shift
        c2w[:, 3] /= 2 * self.scale  # to bound the scene inside [-0.5, 0.5]
        return c2w

    def read_meta(self, split):
        self.rays, self.poses = [], []
        if split == 'test_traj':  # BlendedMVS and TanksAndTemple
            if 'Ignatius' in self.root_dir:
                poses = [np.loadtxt(p) for p in sorted(glob.glob(os.path.join(self.root_dir, 'test_pose/*.txt')))]
            else:
                poses = np.loadtxt(os.path.join(self.root_dir, 'test_traj.txt')).reshape(-1, 4, 4)
            for pose in poses:
                c2w = np.array(pose[:3], dtype=np.float64)
                c2w[:, 0] *= -1  # [left down front] to [right down front]
                self.poses += [self._normalise(c2w)]
        else:
            if split == 'train':
                prefix = '0_'
            elif split == 'trainval':
                prefix = '[0-1]_'
            elif split == 'trainvaltest':
                prefix = '[0-2]_'
            elif split == 'val':
                prefix = '1_'
            elif 'Synthetic' in self.root_dir:
                prefix = '2_'  # test set for synthetic scenes
            elif split == 'test':
                prefix = '1_'  # test set for real scenes
            else:
                raise ValueError(f'{split} split not recognized!')
            img_paths = sorted(glob.glob(os.path.join(self.root_dir, 'rgb', prefix + '*.png')))
            poses = sorted(glob.glob(os.path.join(self.root_dir, 'pose', prefix + '*.txt')))
            for img_path, pose in zip(img_paths, poses):
                self.poses += [self._normalise(np.loadtxt(pose)[:3])]
                img = read_image(img_path, self.img_wh)
                if 'Jade' in self.root_dir or 'Fountain' in self.root_dir:
                    img[np.all(img <= 0.1, axis=-1)] = 1.0  # black background to white
                self.rays += [img]
            self.rays = torch.FloatTensor(np.stack(self.rays))  # (N_images, hw, 3)
        self.poses = torch.FloatTensor(np.stack(self.poses))  # (N_images, 3, 4)
