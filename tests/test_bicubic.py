"""§8f rank 4: the bicubic FPN variant's CSAF upsampling
(train_mobilenetV3_ecagai.py:270,279, F.interpolate(mode="bicubic",
align_corners=True)) on the device vs PyTorch-CPU fp32 — the reference's own
op.  Tolerances: forward 1e-5 relative to the max magnitude (fp32 ulp-level
reordering), backward 1e-5 (summation order); the backward is a gather
(no atomics) and bit-reproducible run to run."""
import pytest
import torch
import torch.nn.functional as F

from _util import rel_err


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,OH,OW,C", [(20, 20, 40, 40, 64), (16, 16, 32, 32, 24),
                                         (5, 7, 13, 9, 3), (1, 4, 3, 8, 8), (8, 8, 8, 8, 16),
                                         (64, 64, 128, 128, 40), (3, 3, 1, 1, 4),
                                         (6, 6, 4, 5, 8)])
def test_bicubic_parity(cuda, H, W, OH, OW, C):
    from jabd_amd import ops
    g = torch.Generator().manual_seed(H * 31 + OW)
    x = torch.randn(2, C, H, W, generator=g)
    wts = torch.randn(2, C, OH, OW, generator=g)
    xr = x.clone().requires_grad_(True)
    ref = F.interpolate(xr, size=[OH, OW], mode="bicubic", align_corners=True)
    (ref * wts).sum().backward()
    xg = x.permute(0, 2, 3, 1).contiguous().to(cuda).requires_grad_(True)
    got = ops.upsample_bicubic(xg, (OH, OW))
    (got * wts.permute(0, 2, 3, 1).to(cuda)).sum().backward()
    assert rel_err(got.permute(0, 3, 1, 2), ref.detach()) < 1e-5
    assert rel_err(xg.grad.permute(0, 3, 1, 2), xr.grad) < 1e-5


@pytest.mark.gpu
def test_bicubic_backward_deterministic(cuda):
    """the backward must not depend on atomics' arrival order."""
    from jabd_amd import ops
    g = torch.Generator().manual_seed(3)
    x = torch.randn(4, 64, 64, 40, generator=g).to(cuda).requires_grad_(True)
    w = torch.randn(4, 128, 128, 40, generator=g).to(cuda)
    grads = []
    for _ in range(3):
        x.grad = None
        (ops.upsample_bicubic(x, (128, 128)) * w).sum().backward()
        grads.append(x.grad.clone())
    assert torch.equal(grads[0], grads[1]) and torch.equal(grads[0], grads[2])
