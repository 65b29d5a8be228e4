"""§8f rank 4: the BECA gate (train_mobilenetV3_ecagai.py:286-316) on the
device vs autograd through a PyTorch-CPU restatement of the reference block
(stdv_channels -> Conv1d -> Hardsigmoid -> x * y).  Forward 1e-5, gradients
1e-4 relative to the max magnitude (the std backward divides by std)."""
import math

import pytest
import torch
import torch.nn.functional as F

from _util import rel_err


def _ref_block(x, w):
    """Reference :276-284 + :301-308 (NCHW)."""
    mean = x.sum(3, keepdim=True).sum(2, keepdim=True) / (x.size(2) * x.size(3))
    var = (x - mean).pow(2).sum(3, keepdim=True).sum(2, keepdim=True) / (x.size(2) * x.size(3))
    y = var.pow(0.5)
    k = w.numel()
    y = F.conv1d(y.squeeze(-1).transpose(-1, -2), w.view(1, 1, k), padding=(k - 1) // 2)
    y = F.hardsigmoid(y.transpose(-1, -2).unsqueeze(-1))
    return x * y.expand_as(x)


def test_beca_kernel_size_rule():
    """eca_block's k = int(|(log2 C + 1) / 2|), bumped to odd (:294-295)."""
    def k(c):
        v = int(abs((math.log(c, 2) + 1) / 2))
        return v if v % 2 else v + 1
    assert [k(c) for c in (16, 40, 64, 128, 256)] == [3, 3, 3, 5, 5]


@pytest.mark.gpu
@pytest.mark.parametrize("B,C,H,W,k", [(2, 64, 40, 40, 3), (3, 40, 20, 20, 3),
                                       (2, 256, 10, 10, 5), (1, 100, 7, 9, 5)])
def test_beca_parity(cuda, B, C, H, W, k):
    from jabd_amd import ops
    g = torch.Generator().manual_seed(C + H)
    x = torch.randn(B, C, H, W, generator=g) * 2 + 0.5
    w = torch.randn(k, generator=g) * 3
    wts = torch.randn(B, C, H, W, generator=g)
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    ref = _ref_block(xr, wr)
    (ref * wts).sum().backward()
    xg = x.permute(0, 2, 3, 1).contiguous().to(cuda).requires_grad_(True)
    wg = w.to(cuda).requires_grad_(True)
    got = ops.beca(xg, wg)
    (got * wts.permute(0, 2, 3, 1).to(cuda)).sum().backward()
    assert rel_err(got.permute(0, 3, 1, 2), ref.detach()) < 1e-5
    assert rel_err(xg.grad.permute(0, 3, 1, 2), xr.grad) < 1e-4
    assert rel_err(wg.grad, wr.grad) < 1e-4
