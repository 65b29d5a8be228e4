"""Index-mapping KATs at the reference's own pyramid sizes.

The reference's FPN / CSAF code resizes with F.interpolate(mode='nearest')
(nets/retinaface_eca_nonlocal.py:70-90, nets/layers.py FPN) and pools with
nn.AdaptiveAvgPool2d((s, s)) for s in (1, 3, 6, 8) (nets/retinaface_eca_
nonlocal.py:37-60, the PSP of the NLM).  At the reference's 840x840 training
size the FPN levels are 105 / 53 / 27 (utils/anchors.py:82-105 KAT: 29518
anchors = 2 (105^2 + 53^2 + 27^2 + 14^2)), sizes where in/out is not an
integer ratio, so these are where an off-by-one bin edge or source row would
show.  The CPU tests pin the closed forms the HIP kernels implement
(csrc/head.hip nearest_src, csrc/modules.hip pool bins) to PyTorch-CPU, the
reference's own implementation of those ops; the GPU tests pin the kernels.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as tF

# (in, out) pairs for nearest up-sampling: 840^2 pyramid, 1024^2 pyramid, the
# 640^2 predict size (80 / 40 / 20) and ragged sizes
NEAREST = [(27, 53), (53, 105), (14, 27), (32, 64), (64, 128), (20, 40), (40, 80), (7, 13),
           (13, 27), (5, 17)]
POOL_IN = [105, 53, 27, 14, 128, 64, 32, 80, 40, 20, 7]
POOL_OUT = [1, 3, 6, 8]


def nearest_src(dst, n_in, n_out):
    """ATen nearest source index: floor(dst * (in / out)) in fp32, clamped."""
    if n_out == n_in:
        return dst
    if n_out == 2 * n_in:
        return dst >> 1
    scale = np.float32(n_in) / np.float32(n_out)
    return min(int(math.floor(np.float32(dst) * scale)), n_in - 1)


def pool_bin(i, n_in, n_out):
    """AdaptiveAvgPool2d bin i: [floor(i*in/out), ceil((i+1)*in/out))."""
    return (i * n_in) // n_out, -((-(i + 1) * n_in) // n_out)


def _index_image(h, w):
    r = torch.arange(h, dtype=torch.float32)[:, None]
    c = torch.arange(w, dtype=torch.float32)[None, :]
    return (r * 1000.0 + c)[None, None]  # exact in fp32 for h, w < 1000


@pytest.mark.parametrize("n_in,n_out", NEAREST)
def test_nearest_closed_form_matches_torch(n_in, n_out):
    x = _index_image(n_in, n_in)
    y = tF.interpolate(x, size=(n_out, n_out), mode="nearest")[0, 0]
    src = [nearest_src(d, n_in, n_out) for d in range(n_out)]
    want = torch.tensor([[r * 1000.0 + c for c in src] for r in src])
    assert torch.equal(y, want)


@pytest.mark.parametrize("n_in", POOL_IN)
@pytest.mark.parametrize("n_out", POOL_OUT)
def test_adaptive_pool_bins_match_torch(n_in, n_out):
    x = _index_image(n_in, n_in).double()
    y = tF.adaptive_avg_pool2d(x, n_out)[0, 0]
    for i in range(n_out):
        r0, r1 = pool_bin(i, n_in, n_out)
        for j in range(n_out):
            c0, c1 = pool_bin(j, n_in, n_out)
            m = x[0, 0, r0:r1, c0:c1].mean()
            assert float(y[i, j]) == pytest.approx(float(m), rel=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("n_in,n_out", NEAREST)
def test_nearest_kernels_match_torch(cuda, n_in, n_out):
    """jabd_upsample_nearest_f32 and the fused upsample+add (FPN merge path)
    reproduce torch's source rows / columns exactly (copies: bit-exact)."""
    from jabd_amd import functional as F
    x = _index_image(n_in, n_in + 3).repeat(2, 4, 1, 1)  # B=2, C=4, ragged W
    want = tF.interpolate(x, size=(n_out, n_out + 5), mode="nearest")
    xh = x.permute(0, 2, 3, 1).contiguous().to(cuda)
    got = F.upsample(xh, n_out, n_out + 5, "nearest").permute(0, 3, 1, 2).cpu()
    assert torch.equal(got, want)
    lat = torch.zeros(2, n_out, n_out + 5, 4, device=cuda)
    got2 = F.upsample_add(xh, lat).permute(0, 3, 1, 2).cpu()
    assert torch.equal(got2, want)


@pytest.mark.gpu
@pytest.mark.parametrize("n_in", [105, 53, 27, 14, 32])
def test_adaptive_pool_kernel_matches_torch(cuda, n_in):
    """jabd_adaptive_pool_f32 (the NLM's PSP, sizes 1/3/6/8) at the 840^2
    pyramid sizes: every bin's mean against torch's adaptive_avg_pool2d."""
    from jabd_amd import functional as F
    g = torch.Generator().manual_seed(n_in)
    x = torch.randn(2, 8, n_in, n_in, generator=g)
    want = torch.cat([tF.adaptive_avg_pool2d(x, s).flatten(2) for s in POOL_OUT], 2)  # [B,C,S]
    got = F.adaptive_pool(x.permute(0, 2, 3, 1).contiguous().to(cuda), POOL_OUT).cpu()
    got = got.permute(0, 2, 1)
    err = float((got - want).abs().max() / want.abs().max())
    assert err < 1e-6, err
