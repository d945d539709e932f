"""Dataset base of the reference's loaders (datasets/base.py:1-35): epoch
length and per-step random ray batches, plus the device-resident ground
truth the native trainer samples from (NGPTrainer.train_step).

Subclasses set K (3,3), directions (h*w,3), img_wh, poses (N,3,4) and rays
(N, h*w, C) with C = 3 (rgb) or 4 (rgb + exposure, HDR data)."""
import numpy as np
import torch
from torch.utils.data import Dataset

TRAIN_STEPS_PER_EPOCH = 1000  # an epoch is 1000 random batches (datasets/base.py:17-19)


class BaseDataset(Dataset):
    def __init__(self, root_dir, split='train', downsample=1.0):
        self.root_dir, self.split, self.downsample = root_dir, split, downsample

    def read_intrinsics(self):
        raise NotImplementedError

    @property
    def _training(self):
        return self.split.startswith('train')

    def __len__(self):
        return TRAIN_STEPS_PER_EPOCH if self._training else len(self.poses)

    def _draw_rays(self):
        """batch_size uniform (image, pixel) pairs: every image
        ('all_images') or one image for the whole batch ('same_image')."""
        n_img, n_pix = len(self.poses), self.img_wh[0] * self.img_wh[1]
        if self.ray_sampling_strategy == 'same_image':
            img = np.random.choice(n_img, 1)[0]
        elif self.ray_sampling_strategy == 'all_images':
            img = np.random.choice(n_img, self.batch_size)
        else:
            raise ValueError(f"unknown ray_sampling_strategy {self.ray_sampling_strategy!r}")
        return img, np.random.choice(n_pix, self.batch_size)

    @staticmethod
    def _with_exposure(sample, colours, exposure):
        sample['rgb'] = colours[..., :3]
        if colours.shape[-1] == 4:  # HDR data carries the exposure as a 4th channel
            sample['exposure'] = exposure
        return sample

    def __getitem__(self, idx):
        if self._training:
            img, pix = self._draw_rays()
            picked = self.rays[img, pix]
            return self._with_exposure({'img_idxs': img, 'pix_idxs': pix}, picked, picked[:, 3:])
        sample = {'pose': self.poses[idx], 'img_idxs': idx}
        if len(self.rays) == 0:  # no ground truth for this split
            return sample
        frame = self.rays[idx]
        return self._with_exposure(sample, frame, frame[0, 3] if frame.shape[-1] == 4 else None)

    def gt_f32(self):
        """(N, h*w, 3) float32 ground truth for NGPTrainer.train_step: the
        training targets exactly as the reference's loss sees them (alpha-
        blended colours are not multiples of 1/255)."""
        return torch.as_tensor(self.rays[..., :3], dtype=torch.float32).contiguous()

    def gt_u8(self):
        """(N, h*w, 3) uint8 ground truth (4x less memory; exact only when the
        colours are multiples of 1/255, e.g. opaque 8-bit images)."""
        return (torch.as_tensor(self.rays[..., :3]).clamp(0, 1) * 255 + 0.5).to(torch.uint8)
