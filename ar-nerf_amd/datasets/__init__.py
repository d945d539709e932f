"""datasets/__init__.py of the reference.  Implemented: 'nerf' (NeRF-synthetic
/ Blender), 'nsvf' (Synthetic_NeRF & co.) and 'colmap' (mip-NeRF 360); the
first two are pinned to fixtures from the reference's own loaders
(tests/test_loaders_golden_cpu.py).  The other loaders of the reference
(colmap_exr, colmap_real_exr, myblender, nerfpp, rtmv: EXR / HDR variants)
are out of scope; asking for one raises."""
from .nerf import NeRFDataset
from .nsvf import NSVFDataset
from .colmap import ColmapDataset


class _Missing:
    def __init__(self, name):
        self.name = name

    def __call__(self, *a, **k):
        raise NotImplementedError(f"dataset '{self.name}' is not implemented in this build (only 'nerf', 'nsvf', 'colmap')")


dataset_dict = {'nerf': NeRFDataset, 'nsvf': NSVFDataset, 'colmap': ColmapDataset}
for _n in ('colmap_exr', 'colmap_real_exr', 'myblender', 'nerfpp', 'rtmv'):
    dataset_dict[_n] = _Missing(_n)
