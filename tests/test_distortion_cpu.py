"""Distortion loss oracle (oracle/vren_oracle.c or_distortion_loss_*, restating
losses.cu:8-173) vs the closed form it computes (Mip-NeRF 360 / DVGO-v2):
  L_ray = sum_i sum_j w_i w_j |t_i - t_j| + 1/3 sum_i w_i^2 delta_i
for sorted t, and its gradient vs autograd of that closed form in fp64."""
import torch

import oracle as O


def _rows(counts, perm_seed=0):
    starts = torch.cumsum(torch.tensor([0] + counts[:-1]), 0)
    ra = torch.stack([torch.arange(len(counts)), starts, torch.tensor(counts)], 1).long()
    g = torch.Generator().manual_seed(perm_seed)
    return ra[torch.randperm(len(counts), generator=g)].contiguous()


def _inputs(counts, seed=0):
    g = torch.Generator().manual_seed(seed)
    N = sum(counts)
    ws = torch.rand(N, generator=g) * 0.2
    deltas = torch.rand(N, generator=g) * 0.01 + 1e-3
    ts = torch.zeros(N)
    s = 0
    for c in counts:  # increasing t along each ray
        ts[s:s + c] = torch.cumsum(torch.rand(c, generator=g) * 0.02 + 1e-3, 0) + 0.5
        s += c
    return ws, deltas, ts


def _closed_form(ws, deltas, ts, ra):
    out = torch.zeros(ra.shape[0], dtype=torch.float64)
    for ray, start, n in ra.tolist():
        w, t, d = ws[start:start + n], ts[start:start + n], deltas[start:start + n]
        out[ray] = (w[:, None] * w[None, :] * (t[:, None] - t[None, :]).abs()).sum() + (w * w * d).sum() / 3
    return out


def test_known_answers():
    # one sample: loss = w^2 delta / 3; two samples: + 2 w0 w1 (t1 - t0)
    ws, d, ts = torch.tensor([0.5, 0.25, 0.5]), torch.tensor([0.03, 0.01, 0.02]), torch.tensor([1.0, 1.5, 2.0])
    ra = torch.tensor([[0, 0, 1], [1, 1, 2]])
    loss, wsi, wtsi = O.distortion_loss_fw(ws, d, ts, ra)
    assert abs(float(loss[0]) - 0.25 * 0.03 / 3) < 1e-8
    want = 2 * 0.25 * 0.5 * 0.5 + (0.0625 * 0.01 + 0.25 * 0.02) / 3
    assert abs(float(loss[1]) - want) < 1e-7
    assert torch.equal(wsi, torch.tensor([0.5, 0.25, 0.75]))
    assert torch.equal(wtsi, torch.tensor([0.5, 0.375, 1.375]))


def test_oracle_matches_closed_form_and_its_gradient():
    counts = [0, 1, 2, 7, 64, 65, 130, 3, 0, 31]
    ws, deltas, ts = _inputs(counts)
    ra = _rows(counts)
    loss, wsi, wtsi = O.distortion_loss_fw(ws, deltas, ts, ra)
    ref = _closed_form(ws.double(), deltas.double(), ts.double(), ra)
    torch.testing.assert_close(loss.double(), ref, rtol=1e-5, atol=1e-8)
    g = torch.rand(len(counts), generator=torch.Generator().manual_seed(3))
    dws = O.distortion_loss_bw(g, wsi, wtsi, ws, deltas, ts, ra)
    w64 = ws.double().requires_grad_()
    (_closed_form(w64, deltas.double(), ts.double(), ra) * g.double()).sum().backward()
    torch.testing.assert_close(dws.double(), w64.grad, rtol=1e-4, atol=1e-7)
