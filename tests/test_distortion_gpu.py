"""vren.distortion_loss_fw/_bw (gfx950) vs the oracle restatement of
losses.cu:8-173: bit-exact (same fp32 operation order, no contraction), on
ragged rows incl. empty / single-sample / >64-sample rows in shuffled order;
the DistortionLoss autograd wrapper (losses.py:7-38) end to end."""
import pytest
import torch

import oracle as O
import vren
from losses import DistortionLoss, NeRFLoss
from test_distortion_cpu import _inputs, _rows

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("seed", [0, 1])
def test_distortion_fw_bw_bit_exact(seed):
    g = torch.Generator().manual_seed(seed)
    counts = [0, 1, 2, 63, 64, 65, 200] + torch.randint(0, 90, (3000,), generator=g).tolist()
    ws, deltas, ts = _inputs(counts, seed)
    ra = _rows(counts, seed)
    ref = O.distortion_loss_fw(ws, deltas, ts, ra)
    out = vren.distortion_loss_fw(ws.to(DEV), deltas.to(DEV), ts.to(DEV), ra.to(DEV))
    for a, b in zip(out, ref):
        assert torch.equal(a.cpu(), b)
    dl = torch.randn(len(counts), generator=g)
    ref_bw = O.distortion_loss_bw(dl, *ref[1:], ws, deltas, ts, ra)
    out_bw = vren.distortion_loss_bw(dl.to(DEV), out[1], out[2], ws.to(DEV), deltas.to(DEV), ts.to(DEV), ra.to(DEV))
    assert torch.equal(out_bw.cpu(), ref_bw)


def test_distortion_autograd_and_nerf_loss():
    counts = [5, 0, 17, 70]
    ws, deltas, ts = _inputs(counts, 4)
    ra = _rows(counts, 4).to(DEV)
    w = ws.to(DEV).requires_grad_()
    loss = DistortionLoss.apply(w, deltas.to(DEV), ts.to(DEV), ra)
    loss.sum().backward()
    ref = O.distortion_loss_fw(ws, deltas, ts, ra.cpu())
    assert torch.equal(loss.detach().cpu(), ref[0])
    assert torch.equal(w.grad.cpu(), O.distortion_loss_bw(torch.ones(4), *ref[1:], ws, deltas, ts, ra.cpu()))
    res = {"rgb": torch.rand(4, 3, device=DEV), "opacity": torch.rand(4, device=DEV), "depth": torch.rand(4, device=DEV),
           "ws": w.detach(), "deltas": deltas.to(DEV), "ts": ts.to(DEV), "rays_a": ra}
    d = NeRFLoss(30, "raw", 0.5, 0.0, lambda_distortion=1e-3)(res, {"rgb": torch.rand(4, 3, device=DEV)})
    torch.testing.assert_close(d["distortion"].cpu(), 1e-3 * ref[0])
