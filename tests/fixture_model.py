"""Test double shaped like the reference NGP (models/networks.py:12-165),
built from the oracle's tcnn-semantics stub modules with the exact seeds and
table override of tests/golden/make_golden.py, so tests can regenerate the
fixtures' parameters instead of storing 45 MB of them."""
import numpy as np
import torch
from torch import nn

import oracle as O
import synthetic as S


def load(name):
    import os
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"{name}.npz"))
    return {k: d[k] for k in d.files}


def checksum(p):
    p = p.detach().double()
    return np.array([p.sum().item(), (p * p).sum().item(), p[:8].sum().item(), p[-8:].sum().item()])


class FixtureModel(nn.Module):
    def __init__(self, scale, seed, amp, sigma_gain=40.0):
        super().__init__()
        self.scale = scale
        self.register_buffer('center', torch.zeros(1, 3))
        self.register_buffer('xyz_min', -torch.ones(1, 3) * scale)
        self.register_buffer('xyz_max', torch.ones(1, 3) * scale)
        self.register_buffer('half_size', (self.xyz_max - self.xyz_min) / 2)
        self.cascades = max(1 + int(np.ceil(np.log2(2 * scale))), 1)
        self.grid_size = 128
        self.register_buffer('density_bitfield',
                             S.packbits_cpu(S.shell_density_grid(128, self.cascades, scale), 0.5))
        b = np.exp(np.log(2048 * scale / 16) / 15)
        self.xyz_encoder = O.tcnn_stub.NetworkWithInputEncoding(
            3, 16, {"otype": "Grid", "type": "Hash", "n_levels": 16, "n_features_per_level": 2,
                    "log2_hashmap_size": 19, "base_resolution": 16, "per_level_scale": b, "interpolation": "Linear"},
            {"otype": "FullyFusedMLP", "activation": "ReLU", "output_activation": "None", "n_neurons": 64,
             "n_hidden_layers": 1})
        self.dir_encoder = O.tcnn_stub.Encoding(3, {"otype": "SphericalHarmonics", "degree": 4})
        self.rgb_net = O.tcnn_stub.Network(32, 3, {"otype": "FullyFusedMLP", "activation": "ReLU",
                                                   "output_activation": "Sigmoid", "n_neurons": 64,
                                                   "n_hidden_layers": 2})
        g = torch.Generator().manual_seed(100 + seed)
        enc = self.xyz_encoder
        with torch.no_grad():
            n = enc.params.numel() - enc.n_mlp
            enc.params[enc.n_mlp:] = (torch.rand(n, generator=g) * 2 - 1) * amp
            enc.params[2048:2048 + 64] *= sigma_gain

    def density(self, x, return_feat=False):
        from models.custom_functions import TruncExp
        x = (x - self.xyz_min) / (self.xyz_max - self.xyz_min)
        h = self.xyz_encoder(x)
        sigmas = TruncExp.apply(h[:, 0].float())
        return (sigmas, h) if return_feat else sigmas

    def forward(self, x, d, **kwargs):
        sigmas, h = self.density(x, return_feat=True)
        d = d / torch.norm(d, dim=1, keepdim=True)
        d = self.dir_encoder((d + 1) / 2)
        rgbs = self.rgb_net(torch.cat([d, h], 1))
        return sigmas, rgbs.float()
