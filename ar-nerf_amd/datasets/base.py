"""datasets/base.py:1-35 of the reference."""
import numpy as np
from torch.utils.data import Dataset


class BaseDataset(Dataset):
    """Length and batch sampling; subclasses fill K, directions, img_wh,
    poses (N,3,4) and rays (N, h*w, 3) ground-truth colours."""

    def __init__(self, root_dir, split='train', downsample=1.0):
        self.root_dir = root_dir
        self.split = split
        self.downsample = downsample

    def read_intrinsics(self):
        raise NotImplementedError

    def __len__(self):
        if self.split.startswith('train'):
            return 1000
        return len(self.poses)

    def __getitem__(self, idx):
        if self.split.startswith('train'):
            if self.ray_sampling_strategy == 'all_images':
                img_idxs = np.random.choice(len(self.poses), self.batch_size)
            elif self.ray_sampling_strategy == 'same_image':
                img_idxs = np.random.choice(len(self.poses), 1)[0]
            pix_idxs = np.random.choice(self.img_wh[0] * self.img_wh[1], self.batch_size)
            rays = self.rays[img_idxs, pix_idxs]
            sample = {'img_idxs': img_idxs, 'pix_idxs': pix_idxs, 'rgb': rays[:, :3]}
            if self.rays.shape[-1] == 4:  # HDR-NeRF data
                sample['exposure'] = rays[:, 3:]
        else:
            sample = {'pose': self.poses[idx], 'img_idxs': idx}
            if len(self.rays) > 0:
                rays = self.rays[idx]
                sample['rgb'] = rays[:, :3]
                if rays.shape[1] == 4:
                    sample['exposure'] = rays[0, 3]
        return sample

    def gt_u8(self):
        """Ground truth as (N, h*w, 3) uint8 for NGPTrainer.train_step (resident in HBM)."""
        return (self.rays[..., :3].clamp(0, 1) * 255 + 0.5).to(dtype=__import__('torch').uint8)
