"""Checkpoint compatibility (utils.py:1-39 of the reference, SURVEY.md §8f
rank 3): a reference-layout Lightning checkpoint (tcnn flat params under
'model.xyz_encoder.params' / 'model.rgb_net.params', buffers, training-only
entries) loads into models.networks.NGP, and NGP state saves back in that
layout; slim_ckpt pops what the reference pops."""
import torch

import utils
from models.networks import NGP


def _ref_ckpt(model, extra=True):
    sd = {'model.' + k: v for k, v in utils.tcnn_state_dict(model).items()}
    if extra:
        sd['model.density_grid'] = torch.rand(model.cascades, 128 ** 3)
        sd['model.grid_coords'] = torch.zeros(128 ** 3, 3, dtype=torch.int32)
        sd['directions'] = torch.zeros(4, 3)
        sd['poses'] = torch.zeros(2, 3, 4)
        sd['val_lpips.net.w'] = torch.zeros(1)
    return {'state_dict': sd, 'epoch': 29}


def test_tcnn_layout_round_trip(tmp_path):
    src = NGP(0.5, seed=7)
    with torch.no_grad():
        src.density_bitfield.random_(0, 255)
    path = str(tmp_path / "epoch=29.ckpt")
    torch.save(_ref_ckpt(src), path)
    dst = NGP(0.5, seed=8)
    assert not torch.equal(dst.params, src.params)
    utils.load_ckpt(dst, path, prefixes_to_ignore=['grid_coords'])
    assert torch.equal(dst.params, src.params)
    assert torch.equal(dst.density_bitfield, src.density_bitfield)
    assert dst.density_grid.shape == (1, 128 ** 3)
    xyz, rgb = dst.tcnn_params()
    assert xyz.numel() == 3072 + 2 * dst.grid.n_entries and rgb.numel() == 7168


def test_slim_ckpt_pops_training_entries(tmp_path):
    m = NGP(0.5)
    path = str(tmp_path / "c.ckpt")
    torch.save(_ref_ckpt(m), path)
    sd = utils.slim_ckpt(path)
    for k in ('directions', 'poses', 'model.density_grid', 'model.grid_coords', 'val_lpips.net.w'):
        assert k not in sd
    assert 'model.xyz_encoder.params' in sd and 'model.density_bitfield' in sd
    assert 'poses' in utils.slim_ckpt(path, save_poses=True)
    # the slimmed dict is itself loadable
    torch.save({'state_dict': sd}, path)
    m2 = NGP(0.5, seed=9)
    utils.load_ckpt(m2, path)
    assert torch.equal(m2.params, m.params)


def test_reference_checkpoint_with_empty_dir_encoder_params(tmp_path):
    """The reference's tcnn SH encoding registers an empty `params` Parameter,
    so its checkpoints hold 'model.dir_encoder.params' of shape [0]."""
    src = NGP(0.5, seed=3)
    ck = _ref_ckpt(src)
    assert ck['state_dict']['model.dir_encoder.params'].shape == (0,)
    path = str(tmp_path / "ref.ckpt")
    torch.save(ck, path)
    dst = NGP(0.5, seed=4)
    utils.load_ckpt(dst, path)
    assert torch.equal(dst.params, src.params)
    ck['state_dict']['model.dir_encoder.params'] = torch.zeros(3)
    torch.save(ck, path)
    import pytest
    with pytest.raises(RuntimeError, match="dir_encoder.params"):
        utils.load_ckpt(NGP(0.5), path)
