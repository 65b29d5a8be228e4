"""Training-graph glue kernels (csrc/glue.hip) against the torch ops they
replace in a training step: torch.cat zero-padding and slicing (window
copies), .t().contiguous() (transpose), .sum over the channel partials
(channel_total), conv_weight_2d (conv_w2d), the heads' weight cat + index_put
(heads_wpack) and the loss sum (weighted_sum3).  Bit-exact: they only move
data, except the channel sum (fixed-order fp32 sum vs torch's, 1e-6)."""
import pytest
import torch


@pytest.mark.gpu
def test_window_copies_pad_crop_offset_scale(cuda):
    from jabd_amd import functional as F
    g = torch.Generator(device=cuda).manual_seed(0)
    w = torch.randn((10, 10, 3, 3), device=cuda, generator=g)
    v = torch.randn(10, device=cuda, generator=g)
    m = torch.randn((7, 8), device=cuda, generator=g)
    s = torch.randn((), device=cuda, generator=g)
    wp = torch.empty((12, 12, 3, 3), device=cuda)
    vp = torch.empty(12, device=cuda)
    crop = torch.empty((10, 10, 3, 3), device=cuda)
    right = torch.empty((1, 7, 3), device=cuda)
    sc = torch.empty((), device=cuda)
    fill = torch.empty((2, 3, 4), device=cuda)
    F.window_copies([(w, wp, 0.0), (v, vp, 1.0), (m.view(1, 7, 8), right, 0.0, 5),
                     (s, sc, 0.0, 0, 2.0), (None, fill, -3.0)])
    F.window_copies([(wp, crop, 0.0)])
    torch.cuda.synchronize()
    ref = torch.zeros((12, 12, 3, 3), device=cuda)
    ref[:10, :10] = w
    assert torch.equal(wp, ref)
    assert torch.equal(vp, torch.cat([v, torch.ones(2, device=cuda)]))
    assert torch.equal(crop, w)
    assert torch.equal(right[0], m[:, 5:])
    assert torch.equal(sc, s * 2.0)
    assert torch.equal(fill, torch.full((2, 3, 4), -3.0, device=cuda))


@pytest.mark.gpu
def test_pad_fn_gradient_is_the_crop(cuda):
    from jabd_amd import train as T
    w = torch.randn((10, 12, 5, 5), device=cuda, requires_grad=True)
    b = torch.randn(10, device=cuda, requires_grad=True)
    rm = torch.randn(10, device=cuda)
    wp, bp, rmp = T._padded([(w, (12, 12, 5, 5), 0.0), (b, (12,), 0.0), (rm, (12,), 0.0)])
    assert not rmp.requires_grad
    gw = torch.randn_like(wp)
    gb = torch.randn_like(bp)
    torch.autograd.backward([wp, bp], [gw, gb])
    assert torch.equal(w.grad, gw[:10])
    assert torch.equal(b.grad, gb[:10])


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(9, 16), (25, 120), (1, 3)])
def test_transpose(cuda, shape):
    from jabd_amd import functional as F
    x = torch.randn(shape, device=cuda)
    assert torch.equal(F.transpose(x), x.t().contiguous())


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(2, 16, 16, 32), (3, 7, 9, 12), (1, 128, 128, 40),
                                   (32, 64, 64, 40), (4, 16, 16, 200), (5, 8, 8, 3)])
def test_channel_total(cuda, shape):
    """Fixed-order parallel reduction: within 1e-6 of fp64, bitwise repeatable
    (2048 partial rows at the C4 bias-gradient shape, C > 64 over several
    workgroups, C not a multiple of 4)."""
    from jabd_amd import functional as F
    x = torch.randn(shape, device=cuda)
    ref = x.double().sum((0, 1, 2))
    got = F.channel_total(x)
    assert float((got.double() - ref).abs().max()) <= 1e-6 * float(x.abs().sum((0, 1, 2)).max())
    assert torch.equal(got, F.channel_total(x))


@pytest.mark.gpu
def test_conv_w2d_matches_conv_weight_2d(cuda):
    from jabd_amd import functional as F
    from jabd_amd._lib import call
    w = torch.randn((16, 3, 3, 3), device=cuda)
    out = torch.empty((27, 16), device=cuda)
    call("jabd_conv_w2d_f32", w.data_ptr(), 16, 3, 9, out.data_ptr(), None)
    torch.cuda.synchronize()
    assert torch.equal(out, F.conv_weight_2d(w).contiguous())


@pytest.mark.gpu
@pytest.mark.parametrize("layout", [None, (20, 10, 12)])
def test_heads_wpack_round_trip(cuda, layout):
    """Pack: the cat of the three weights with zero columns at the padded SSH
    channels (the former cat + new_zeros + index_put); unpack: the column
    gather of a weight gradient (the former dW[:, idx])."""
    from jabd_amd._lib import call
    C = 40
    half, q, qp = layout if layout else (C, 0, 0)
    Cf = half + 2 * qp if layout else C
    ws = [torch.randn((r, C, 1, 1), device=cuda) for r in (8, 4, 20)]
    bs = [torch.randn(r, device=cuda) for r in (8, 4, 20)]
    wt = torch.empty((32, Cf), device=cuda)
    bias = torch.empty(32, device=cuda)
    call("jabd_heads_wpack_f32", ws[0].data_ptr(), ws[1].data_ptr(), ws[2].data_ptr(),
         bs[0].data_ptr(), bs[1].data_ptr(), bs[2].data_ptr(), C, half, q, qp, wt.data_ptr(),
         Cf, bias.data_ptr(), 0, None)
    full = torch.cat([w.view(-1, C) for w in ws])
    idx = torch.arange(C, device=cuda)
    if layout:
        idx = torch.cat([idx[:half + q], idx[half + q:] + (qp - q)])
    ref = torch.zeros((32, Cf), device=cuda)
    ref[:, idx] = full
    torch.cuda.synchronize()
    assert torch.equal(wt, ref)
    assert torch.equal(bias, torch.cat(bs))
    dW = torch.randn((32, Cf), device=cuda)
    g3 = [torch.full((r, C, 1, 1), float("nan"), device=cuda) for r in (8, 4, 20)]
    call("jabd_heads_wpack_f32", g3[0].data_ptr(), g3[1].data_ptr(), g3[2].data_ptr(),
         None, None, None, C, half, q, qp, dW.data_ptr(), Cf, None, 1, None)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat([t.view(-1, C) for t in g3]), dW[:, idx])


@pytest.mark.gpu
def test_weighted_loss_sum(cuda):
    from jabd_amd import parallel
    r, c, lm = (torch.tensor(v, device=cuda, requires_grad=True) for v in (0.7, 1.3, 2.9))
    loss = parallel._WeightedLossFn.apply(r, c, lm, 2.0)
    assert torch.equal(loss, 2.0 * r.detach() + c.detach() + lm.detach())
    torch.autograd.backward(loss, parallel._one(cuda))
    assert float(r.grad) == 2.0 and float(c.grad) == 1.0 and float(lm.grad) == 1.0
