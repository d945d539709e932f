"""The oracle's d sigma / d x (oracle.density_input_grad, autograd through the
tcnn-semantics hash grid) against central finite differences of the same
field evaluated in fp64 (no fp16 rounding of activations): the directions
agree (cos >= 0.999 for >= 99% of points).  The finest level's cells are
~5e-4 wide, so the difference step must be far smaller (1e-7) to stay inside
one cell."""
import torch

import oracle as O


def _sig64(f, xx):
    idx, _ = O.hash_corners(f.spec, xx.float(), f.xyz_min, f.xyz_max)
    tab = f.xyz_params.detach()[f.n_dens:].half().double().view(-1, 2)
    x01 = (xx - f.xyz_min.double()) / (f.xyz_max.double() - f.xyz_min.double())
    feats = []
    for l in range(f.spec.L):
        p = x01 * float(f.spec.scales[l]) + 0.5
        fr = p - torch.floor(p)
        w = torch.stack([(fr[:, 0] if c & 1 else 1 - fr[:, 0]) * (fr[:, 1] if c & 2 else 1 - fr[:, 1]) *
                         (fr[:, 2] if c & 4 else 1 - fr[:, 2]) for c in range(8)], 1)
        feats.append((w[:, :, None] * tab[idx[:, l, :].long()]).sum(1))
    enc = torch.cat(feats, 1)
    Ws, _ = O.mlp_layers(f.xyz_params.detach()[:f.n_dens].double(), (32, 64, 16))
    h = torch.relu(enc @ Ws[0].half().double().t()) @ Ws[1].half().double().t()
    return torch.exp(h[:, 0])


def test_oracle_input_grad_matches_finite_differences():
    torch.manual_seed(0)
    f = O.OracleNGPField(0.5, table_init=0.5)
    x = (torch.rand(256, 3) * 2 - 1) * 0.45
    g = O.density_input_grad(f.xyz_params.detach(), f.n_dens, f.spec, x, f.xyz_min, f.xyz_max).double()
    eps, E = 1e-7, torch.eye(3, dtype=torch.float64)
    fd = torch.stack([(_sig64(f, x.double() + eps * E[d]) - _sig64(f, x.double() - eps * E[d])) / (2 * eps)
                      for d in range(3)], 1)
    cos = (torch.nn.functional.normalize(fd, dim=1) * torch.nn.functional.normalize(g, dim=1)).sum(1)
    assert float((cos >= 0.999).double().mean()) >= 0.99
    assert float(cos.median()) > 0.99999
