"""datasets/colmap.py:15-166 of the reference: COLMAP scenes (mip-NeRF 360
'garden' & co.): intrinsics from sparse/0/cameras.bin (camera 1), c2w from
images.bin sorted by image name, centred on the point cloud's average pose
(center_poses) and scaled so the closest camera is at distance 1; every 8th
image is the test set.  HDR-NeRF variants are not supported here."""
import os

import numpy as np
import torch

from .base import BaseDataset
from .color_utils import read_image
from .colmap_utils import read_cameras_binary, read_images_binary, read_points3d_binary
from .ray_utils import center_poses, create_spheric_poses, get_ray_directions


class ColmapDataset(BaseDataset):
    def __init__(self, root_dir, split='train', downsample=1.0, **kwargs):
        super().__init__(root_dir, split, downsample)
        self.read_intrinsics()
        if kwargs.get('read_meta', True):
            self.read_meta(split, **kwargs)

    def read_intrinsics(self):
        cam = read_cameras_binary(os.path.join(self.root_dir, 'sparse/0/cameras.bin'))[1]
        h, w = int(cam.height * self.downsample), int(cam.width * self.downsample)
        self.img_wh = (w, h)
        if cam.model == 'SIMPLE_RADIAL':
            fx = fy = cam.params[0] * self.downsample
            cx, cy = cam.params[1] * self.downsample, cam.params[2] * self.downsample
        elif cam.model in ('PINHOLE', 'OPENCV'):
            fx, fy = cam.params[0] * self.downsample, cam.params[1] * self.downsample
            cx, cy = cam.params[2] * self.downsample, cam.params[3] * self.downsample
        else:
            raise ValueError(f"Please parse the intrinsics for camera model {cam.model}!")
        self.K = torch.FloatTensor([[fx, 0, cx], [0, fy, cy], [0, 0, 1]])
        self.directions = get_ray_directions(h, w, self.K)

    def read_meta(self, split, **kwargs):
        if 'HDR-NeRF' in self.root_dir:
            raise NotImplementedError("HDR-NeRF data (exposure channel) is out of scope")
        imdata = read_images_binary(os.path.join(self.root_dir, 'sparse/0/images.bin'))
        img_names = [imdata[k].name for k in imdata]
        perm = np.argsort(img_names)
        folder = f'images_{int(1 / self.downsample)}' if '360_v2' in self.root_dir and self.downsample < 1 \
            else 'images'
        img_paths = [os.path.join(self.root_dir, folder, name) for name in sorted(img_names)]
        bottom = np.array([[0, 0, 0, 1.]])
        w2c = np.stack([np.concatenate([np.concatenate([imdata[k].qvec2rotmat(), imdata[k].tvec.reshape(3, 1)], 1),
                                        bottom], 0) for k in imdata], 0)
        poses = np.linalg.inv(w2c)[perm, :3]  # (N_images, 3, 4) cam2world
        pts3d = read_points3d_binary(os.path.join(self.root_dir, 'sparse/0/points3D.bin'))
        pts3d = np.array([pts3d[k].xyz for k in pts3d])
        self.poses, self.pts3d, pose_avg = center_poses(poses, pts3d)
        scale = np.linalg.norm(self.poses[..., 3], axis=-1).min()
        self.poses[..., 3] /= scale
        self.pts3d /= scale
        self.blender_trans = np.eye(4)
        self.blender_trans[:3, :] = pose_avg
        self.blender_scale = scale
        self.rays = []
        if split == 'test_traj':
            self.poses = torch.FloatTensor(create_spheric_poses(1.2, self.poses[:, 1, 3].mean()))
            return
        if split == 'train':
            keep = [i for i in range(len(img_paths)) if i % 8 != 0]
        elif split == 'test':
            keep = [i for i in range(len(img_paths)) if i % 8 == 0]
        else:
            keep = list(range(len(img_paths)))
        img_paths = [img_paths[i] for i in keep]
        self.poses = np.array([self.poses[i] for i in keep])
        self.rays = torch.stack([torch.FloatTensor(read_image(p, self.img_wh, blend_a=False)) for p in img_paths])
        self.poses = torch.FloatTensor(self.poses)
