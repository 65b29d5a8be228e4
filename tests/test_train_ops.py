"""Per-op backward parity of the training Functions (jabd_amd/train.py)
against autograd of the same math in PyTorch-CPU float64 (test-only
reference).  Tolerance: max-abs error <= 1e-4 of each tensor's magnitude."""
import pytest
import torch
import torch.nn.functional as tF

from _util import rel_err

TOL = 1e-4


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def _nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def _check(got_list, ref_list, names):
    for g, r, n in zip(got_list, ref_list, names):
        assert g is not None, n
        e = rel_err(g, r)
        assert e < TOL, f"{n}: rel err {e:.2e}"


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,k,s,h", [(16, 64, 1, 1, 12), (40, 40, 3, 1, 9), (256, 128, 3, 1, 4),
                                            (64, 64, 3, 2, 11), (256, 512, 1, 2, 8),
                                            (12, 10, 3, 1, 7), (1024, 256, 1, 1, 4),
                                            (128, 128, 3, 2, 10), (64, 96, 3, 2, 9),
                                            (96, 64, 1, 2, 7)])
def test_convfn_grads(cuda, cin, cout, k, s, h):
    from jabd_amd.train import ConvFn
    g = torch.Generator().manual_seed(cin + k)
    x = torch.randn(2, cin, h, h + 1, generator=g)
    w = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    dy_seed = torch.Generator().manual_seed(7)
    xr, wr = x.double().requires_grad_(), w.double().requires_grad_()
    y = tF.conv2d(xr, wr, None, s, k // 2)
    dy = torch.randn(y.shape, generator=dy_seed, dtype=torch.float64)
    (y * dy).sum().backward()
    xg = _nhwc(x).to(cuda).requires_grad_()
    wg = torch.nn.Parameter(w.to(cuda))
    yg = ConvFn.apply(xg, wg, None, s, k // 2, False)
    assert rel_err(_nchw(yg.detach()), y.detach()) < TOL
    (yg * _nhwc(dy.float()).to(cuda)).sum().backward()
    _check([_nchw(xg.grad), wg.grad], [xr.grad, wr.grad], ["dx", "dw"])


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,k,s,h,w", [(3, 16, 3, 2, 64, 200), (3, 16, 3, 2, 37, 51),
                                              (3, 8, 3, 1, 20, 70), (1, 16, 5, 2, 33, 129),
                                              (3, 64, 7, 2, 40, 44), (3, 64, 7, 2, 1, 3),
                                              (3, 64, 7, 2, 131, 261), (3, 64, 7, 2, 256, 256)])
def test_convfn_nchw_input_wgrad(cuda, cin, cout, k, s, h, w):
    """Forward and weight gradient of a conv on the NCHW network input: the
    MobileNetV3 stem shape (3x3/s2, 3 -> 16; stem_wgrad_kernel), widths and
    heights that are not multiples of the 64-pixel segment, and the R50 7x7
    stem (stem7.hip: 4x64 output tiles, a 1x2 output, ragged tiles in both
    directions, several persistent tiles per workgroup)."""
    from jabd_amd.train import ConvFn
    g = torch.Generator().manual_seed(cin * 100 + h)
    x = torch.randn(2, cin, h, w, generator=g) * 50
    wt = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    wr = wt.double().requires_grad_()
    y = tF.conv2d(x.double(), wr, None, s, k // 2)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (y * dy).sum().backward()
    wg = torch.nn.Parameter(wt.to(cuda))
    yg = ConvFn.apply(x.to(cuda), wg, None, s, k // 2, True)
    assert rel_err(_nchw(yg.detach()), y.detach()) < TOL
    (yg * _nhwc(dy.float()).to(cuda)).sum().backward()
    _check([wg.grad], [wr.grad], ["dw"])


@pytest.mark.gpu
@pytest.mark.parametrize("b,h,w", [(1, 64, 64), (2, 45, 300), (3, 129, 67)])
def test_stem7_eval_bias_relu(cuda, b, h, w):
    """The R50 stem's eval form (folded BN bias + ReLU in the stem7 epilogue,
    jabd_amd.functional.conv) against float64 conv2d + bias + relu."""
    from jabd_amd import functional as F
    g = torch.Generator().manual_seed(h * w)
    conv = torch.nn.Conv2d(3, 64, 7, 2, 3)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) / 147 ** 0.5)
        conv.bias.copy_(torch.randn(64, generator=g))
    x = torch.randn(b, 3, h, w, generator=g) * 30
    ref = tF.relu(tF.conv2d(x.double(), conv.weight.double(), conv.bias.double(), 2, 3))
    pk = F.pack_conv(conv.to(cuda))
    y = F.conv(x.to(cuda), pk, stride=2, pad=3, act="relu", nchw_in=True)
    assert rel_err(_nchw(y), ref) < TOL


@pytest.mark.gpu
@pytest.mark.parametrize("c,cout,k,gate,h", [(40, 40, 1, "sigmoid", 8), (256, 128, 3, "sigmoid", 4),
                                             (72, 24, 1, "hsigmoid", 10), (2048, 256, 1, "sigmoid", 3)])
def test_ecaconvfn_grads(cuda, c, cout, k, gate, h):
    from jabd_amd.train import EcaConvFn
    from oracle.model_ref import eca_kernel_size
    g = torch.Generator().manual_seed(c)
    x = torch.randn(2, c, h, h, generator=g)
    ke = eca_kernel_size(c)
    w1 = torch.randn(1, 1, ke, generator=g)
    w = torch.randn(cout, c, k, k, generator=g) / (c * k * k) ** 0.5
    xr, w1r, wr = (t.double().requires_grad_() for t in (x, w1, w))
    yv = xr.mean(dim=(2, 3))
    z = tF.conv1d(yv.unsqueeze(1), w1r, padding=(ke - 1) // 2).squeeze(1)
    sc = torch.sigmoid(z) if gate == "sigmoid" else tF.hardsigmoid(z)
    y = tF.conv2d(xr * sc[:, :, None, None], wr, None, 1, k // 2)
    dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(3), dtype=torch.float64)
    (y * dy).sum().backward()
    xg = _nhwc(x).to(cuda).requires_grad_()
    w1g = torch.nn.Parameter(w1.to(cuda))
    wg = torch.nn.Parameter(w.to(cuda))
    yg = EcaConvFn.apply(xg, w1g, wg, 1, k // 2, gate)
    assert rel_err(_nchw(yg.detach()), y.detach()) < TOL
    (yg * _nhwc(dy.float()).to(cuda)).sum().backward()
    _check([_nchw(xg.grad), w1g.grad, wg.grad], [xr.grad, w1r.grad, wr.grad], ["dx", "dw1d", "dw"])


@pytest.mark.gpu
@pytest.mark.parametrize("c,act,res", [(40, "relu", False), (24, "hswish", True), (2048, "relu", True),
                                       (256, "leaky", False), (12, "none", False)])
def test_bnactfn_grads(cuda, c, act, res):
    from jabd_amd.train import BnActFn
    g = torch.Generator().manual_seed(c)
    x = torch.randn(3, c, 5, 6, generator=g) * 2 + 1
    gam = 1 + 0.2 * torch.randn(c, generator=g)
    bet = 0.1 * torch.randn(c, generator=g)
    r = torch.randn(3, c, 5, 6, generator=g) if res else None
    xr, gr, br = (t.double().requires_grad_() for t in (x, gam, bet))
    rr = r.double().requires_grad_() if res else None
    rm, rv = torch.zeros(c, dtype=torch.float64), torch.ones(c, dtype=torch.float64)
    z = tF.batch_norm(xr, rm, rv, gr, br, True, 0.1, 1e-5)
    if res:
        z = z + rr
    y = {"relu": tF.relu, "hswish": tF.hardswish, "leaky": lambda t: tF.leaky_relu(t, 0.1),
         "none": lambda t: t}[act](z)
    dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(4), dtype=torch.float64)
    (y * dy).sum().backward()
    xg = _nhwc(x).to(cuda).requires_grad_()
    gg, bg = (torch.nn.Parameter(t.to(cuda)) for t in (gam, bet))
    rg = _nhwc(r).to(cuda).requires_grad_() if res else None
    rmg, rvg = torch.zeros(c, device=cuda), torch.ones(c, device=cuda)
    yg = BnActFn.apply(xg, gg, bg, rg, rmg, rvg, act, 0.1, 0.1, 1e-5)
    assert rel_err(_nchw(yg.detach()), y.detach()) < TOL
    (yg * _nhwc(dy.float()).to(cuda)).sum().backward()
    got = [_nchw(xg.grad), gg.grad, bg.grad] + ([_nchw(rg.grad)] if res else [])
    ref = [xr.grad, gr.grad, br.grad] + ([rr.grad] if res else [])
    _check(got, ref, ["dx", "dgamma", "dbeta", "dres"])
    assert rel_err(rmg, rm) < TOL and rel_err(rvg, rv) < TOL


@pytest.mark.gpu
@pytest.mark.parametrize("c,k,s,h", [(16, 3, 1, 9), (64, 3, 2, 10), (72, 5, 2, 11), (120, 5, 1, 6),
                                     # tall maps: the 3x3 weight gradient walks chunks of
                                     # 5 / 4 output rows (train.hip dw_wgrad_rows_kernel),
                                     # the last chunk short
                                     (16, 3, 1, 703), (24, 3, 2, 701)])
def test_dwconvfn_grads(cuda, c, k, s, h):
    from jabd_amd.train import DwConvFn
    g = torch.Generator().manual_seed(c + k)
    x = torch.randn(2, c, h, h + 2, generator=g)
    w = torch.randn(c, 1, k, k, generator=g) / k
    xr, wr = x.double().requires_grad_(), w.double().requires_grad_()
    y = tF.conv2d(xr, wr, None, s, k // 2, 1, c)
    dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(2), dtype=torch.float64)
    (y * dy).sum().backward()
    xg = _nhwc(x).to(cuda).requires_grad_()
    wg = torch.nn.Parameter(w.to(cuda))
    yg = DwConvFn.apply(xg, wg, s)
    assert rel_err(_nchw(yg.detach()), y.detach()) < TOL
    (yg * _nhwc(dy.float()).to(cuda)).sum().backward()
    _check([_nchw(xg.grad), wg.grad], [xr.grad, wr.grad], ["dx", "dw"])


@pytest.mark.gpu
@pytest.mark.parametrize("C,hs,h", [(40, 4, 8), (256, 2, 4), (40, 27, 53), (40, 6, 12)])
def test_nlmfn_grads(cuda, C, hs, h):
    from jabd_amd.train import NlmFn
    from oracle.model_ref import Ctx, nlm
    g = torch.Generator().manual_seed(C + h)
    src = torch.randn(2, C, hs, hs, generator=g)
    lat = torch.randn(2, C, h, h, generator=g)
    P = {"n.f_query.weight": torch.randn(4, C, 1, 1, generator=g) / C ** 0.5,
         "n.f_query.bias": 0.1 * torch.randn(4, generator=g),
         "n.f_key.weight": torch.randn(4, C, 1, 1, generator=g) / C ** 0.5,
         "n.f_key.bias": 0.1 * torch.randn(4, generator=g),
         "n.f_value.weight": torch.randn(4, C, 1, 1, generator=g) / C ** 0.5,
         "n.f_value.bias": 0.1 * torch.randn(4, generator=g),
         "n.W.weight": torch.randn(C, 4, 1, 1, generator=g) / 2,
         "n.W.bias": 0.1 * torch.randn(C, generator=g)}
    Pr = {k: v.double().requires_grad_() for k, v in P.items()}
    sr, lr = src.double().requires_grad_(), lat.double().requires_grad_()
    up = tF.interpolate(sr, size=[h, h], mode="nearest")
    y = lr + nlm(Ctx(Pr), up, "n.")
    dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(8), dtype=torch.float64)
    (y * dy).sum().backward()
    Pg = {k: torch.nn.Parameter(v.to(cuda)) for k, v in P.items()}
    sg, lg = _nhwc(src).to(cuda).requires_grad_(), _nhwc(lat).to(cuda).requires_grad_()
    order = ["n.f_query.weight", "n.f_query.bias", "n.f_key.weight", "n.f_key.bias",
             "n.f_value.weight", "n.f_value.bias", "n.W.weight", "n.W.bias"]
    yg = NlmFn.apply(sg, lg, *[Pg[k] for k in order], (1, 4, 8, 12))
    assert rel_err(_nchw(yg.detach()), y.detach()) < TOL
    (yg * _nhwc(dy.float()).to(cuda)).sum().backward()
    got = [_nchw(sg.grad), _nchw(lg.grad)] + [Pg[k].grad for k in order if k != "n.f_key.bias"]
    ref = [sr.grad, lr.grad] + [Pr[k].grad for k in order if k != "n.f_key.bias"]
    _check(got, ref, ["dsrc", "dlat"] + [k for k in order if k != "n.f_key.bias"])


@pytest.mark.gpu
@pytest.mark.parametrize("C", [40, 256])
def test_headsfn_grads(cuda, C):
    from jabd_amd.train import HeadsFn
    g = torch.Generator().manual_seed(C)
    feats = [torch.randn(2, C, s, s, generator=g) for s in (8, 4, 2)]
    wb = []
    for _ in range(3):
        for n in (8, 4, 20):
            wb += [torch.randn(n, C, 1, 1, generator=g) / C ** 0.5, 0.1 * torch.randn(n, generator=g)]
    fr = [f.double().requires_grad_() for f in feats]
    wr = [t.double().requires_grad_() for t in wb]
    outs = []
    for kind, (k, off) in enumerate(((4, 0), (2, 2), (10, 4))):
        parts = []
        for i, f in enumerate(fr):
            o = tF.conv2d(f, wr[6 * i + off], wr[6 * i + off + 1]).permute(0, 2, 3, 1)
            parts.append(o.reshape(2, -1, k))
        outs.append(torch.cat(parts, 1))
    dys = [torch.randn(o.shape, generator=torch.Generator().manual_seed(i), dtype=torch.float64)
           for i, o in enumerate(outs)]
    sum((o * d).sum() for o, d in zip(outs, dys)).backward()
    fg = [_nhwc(f).to(cuda).requires_grad_() for f in feats]
    wg = [torch.nn.Parameter(t.to(cuda)) for t in wb]
    og = HeadsFn.apply(*fg, (None, None, None), *wg)
    for o, r in zip(og, outs):
        assert rel_err(o.detach(), r.detach()) < TOL
    sum((o * d.float().to(cuda)).sum() for o, d in zip(og, dys)).backward()
    _check([_nchw(f.grad) for f in fg] + [w.grad for w in wg],
           [f.grad for f in fr] + [w.grad for w in wr], [f"t{i}" for i in range(21)])


@pytest.mark.gpu
def test_maxpoolfn_grads(cuda):
    from jabd_amd.train import MaxPoolFn
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 64, 9, 10, generator=g)
    xr = x.double().requires_grad_()
    y = tF.max_pool2d(xr, 3, 2, 1)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (y * dy).sum().backward()
    xg = _nhwc(x).to(cuda).requires_grad_()
    yg = MaxPoolFn.apply(xg)
    assert rel_err(_nchw(yg.detach()), y.detach()) < TOL
    (yg * _nhwc(dy.float()).to(cuda)).sum().backward()
    _check([_nchw(xg.grad)], [xr.grad], ["dx"])


@pytest.mark.gpu
@pytest.mark.parametrize("B,C,nblk,k,gate", [(3, 16, 1024, 3, "hsigmoid"), (2, 72, 256, 3, "hsigmoid"),
                                             (2, 672, 16, 5, "hsigmoid"), (2, 960, 4, 5, "sigmoid"),
                                             (1, 40, 7, 3, "sigmoid"), (2, 250, 33, 5, "sigmoid")])
def test_eca_gate_from_partials(cuda, B, C, nblk, k, gate):
    """ECA gate from tile partial sums (AdaptiveAvgPool -> Conv1d(k, pad (k-1)/2,
    no bias) -> (hard)sigmoid, nets/mobilenetV3.py:94-112) vs torch fp64: the
    quad-vectorised kernel (C % 4 == 0, windows of 248 channels past C = 248)
    and the per-channel fallback (C = 250)."""
    from jabd_amd import functional as F
    g = torch.Generator().manual_seed(C + nblk)
    part = torch.randn(B, nblk, C, generator=g)
    w = torch.randn(k, generator=g) * 0.5
    hw = nblk * 64
    mean = part.double().sum(1) / hw
    y = torch.nn.functional.conv1d(mean[:, None, :], w.double()[None, None, :], padding=(k - 1) // 2)[:, 0]
    want = torch.sigmoid(y) if gate == "sigmoid" else torch.nn.functional.hardsigmoid(y)
    got, m = F.eca_gate(part.to(cuda), hw, w.to(cuda), gate, return_mean=True)
    assert float((got.cpu().double() - want).abs().max()) < 1e-6
    assert float((m.cpu().double() - mean).abs().max() / mean.abs().max()) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("B,h,w,E,cout", [(3, 32, 48, 64, 24), (3, 32, 48, 480, 112),
                                          (2, 16, 16, 672, 160), (4, 8, 8, 120, 40)])
def test_wgrad_eca(cuda, B, h, w, E, cout):
    """jabd_conv_wgrad_eca_f32: dW of conv1x1(d * s) and ds = sum_hw(da * d),
    da = dp W, from one GEMM over image-aligned chunks, vs float64."""
    from jabd_amd.train import _wgrad_eca
    g = torch.Generator().manual_seed(E)
    d = torch.randn(B, h, w, E, generator=g, dtype=torch.float64)
    dp = torch.randn(B, h, w, cout, generator=g, dtype=torch.float64)
    s = torch.rand(B, E, generator=g, dtype=torch.float64)
    W = torch.randn(cout, E, 1, 1, generator=g, dtype=torch.float64) / E ** 0.5
    dw_ref = torch.einsum("bhwc,bhwn,bc->nc", d, dp, s)
    ds_ref = torch.einsum("bhwn,nc,bhwc->bc", dp, W[:, :, 0, 0], d)
    r = _wgrad_eca(d.float().to(cuda), dp.float().to(cuda), W.float().to(cuda),
                   s.float().to(cuda))
    assert r is not None
    dw, ds = r
    _check([dw[:, :, 0, 0], ds], [dw_ref, ds_ref], ["dw", "ds"])


@pytest.mark.gpu
@pytest.mark.parametrize("c,k,h,w", [(480, 3, 32, 48), (120, 5, 32, 64), (120, 5, 32, 32),
                                     (64, 3, 16, 64), (40, 5, 8, 72)])
def test_dwconvfn_grads_wide(cuda, c, k, h, w):
    """Depthwise backward on wider maps (several W strips per row)."""
    from jabd_amd.train import DwConvFn
    g = torch.Generator().manual_seed(c + k)
    x = torch.randn(3, c, h, w, generator=g)
    wt = torch.randn(c, 1, k, k, generator=g) / k
    xr, wr = x.double().requires_grad_(), wt.double().requires_grad_()
    y = tF.conv2d(xr, wr, None, 1, k // 2, 1, c)
    dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(2), dtype=torch.float64)
    (y * dy).sum().backward()
    xg = _nhwc(x).to(cuda).requires_grad_()
    wg = torch.nn.Parameter(wt.to(cuda))
    yg = DwConvFn.apply(xg, wg, 1)
    assert rel_err(_nchw(yg.detach()), y.detach()) < TOL
    (yg * _nhwc(dy.float()).to(cuda)).sum().backward()
    _check([_nchw(xg.grad), wg.grad], [xr.grad, wr.grad], ["dx", "dw"])


@pytest.mark.gpu
@pytest.mark.parametrize("c,act,h,w", [(480, "hswish", 32, 48), (120, "relu", 32, 64),
                                       (120, "relu", 32, 32)])
def test_bnactfn_grads_wide(cuda, c, act, h, w):
    from jabd_amd.train import BnActFn
    g = torch.Generator().manual_seed(c)
    x = torch.randn(3, c, h, w, generator=g) * 2 + 1
    gam = 1 + 0.2 * torch.randn(c, generator=g)
    bet = 0.1 * torch.randn(c, generator=g)
    xr, gr, br = (t.double().requires_grad_() for t in (x, gam, bet))
    rm, rv = torch.zeros(c, dtype=torch.float64), torch.ones(c, dtype=torch.float64)
    z = tF.batch_norm(xr, rm, rv, gr, br, True, 0.1, 1e-5)
    y = {"relu": tF.relu, "hswish": tF.hardswish}[act](z)
    dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(4), dtype=torch.float64)
    (y * dy).sum().backward()
    xg = _nhwc(x).to(cuda).requires_grad_()
    gg, bg = (torch.nn.Parameter(t.to(cuda)) for t in (gam, bet))
    rmg, rvg = torch.zeros(c, device=cuda), torch.ones(c, device=cuda)
    yg = BnActFn.apply(xg, gg, bg, None, rmg, rvg, act, 0.1, 0.1, 1e-5)
    assert rel_err(_nchw(yg.detach()), y.detach()) < TOL
    (yg * _nhwc(dy.float()).to(cuda)).sum().backward()
    _check([_nchw(xg.grad), gg.grad, bg.grad], [xr.grad, gr.grad, br.grad],
           ["dx", "dgamma", "dbeta"])


def _act_masked(z, zmask, act):
    """act(z) in float64 whose derivative takes its region from zmask (the
    HIP kernel's own fp32 pre-activation), PyTorch's *_backward conventions:
    relu' = [z > 0]; hardswish' = 0 below -3, z/3 + 1/2 on [-3, 3], 1 above."""
    if act == "relu":
        return torch.where(zmask > 0, z, z * 0)
    return torch.where(zmask < -3, z * 0, torch.where(zmask <= 3, z * (z + 3) / 6, z))


@pytest.mark.gpu
@pytest.mark.parametrize("c,k,s,bhw,act", [(64, 3, 2, (4, 64, 48), "relu"), (72, 5, 1, (3, 37, 29), "relu"),
                                           (240, 3, 2, (2, 30, 34), "hswish"),
                                           (480, 3, 1, (3, 32, 48), "hswish"), (16, 3, 1, (2, 9, 5), "relu"),
                                           # tall maps: more rows than partial blocks; stride 2
                                           # with an odd height (chunks starting on odd rows)
                                           (16, 3, 1, (2, 5000, 40), "relu"),
                                           (16, 3, 2, (2, 8201, 40), "hswish")])
@pytest.mark.parametrize("recompute", [True, False])
def test_dw_dgrad_bn_fused(cuda, c, k, s, bhw, act, recompute, monkeypatch):
    """MNv3 block backward through bn1 + act -> depthwise conv: the fused
    depthwise data gradient + bn1 backward partials (jabd_dw_dgrad_bn_bwd_f32)
    against the two-pass form (jabd_dw_dgrad_f32 then jabd_bn_act_bwd_f32):
    the depthwise gradient bit-identical, dgamma / dbeta / dx within fp32
    reassociation of the partial sums; and both against float64 autograd.
    recompute: de not stored, recomputed by a second depthwise pass that
    writes dx (dz == NULL).

    The float64 reference takes its activation region from the HIP
    backward's own fp32 pre-activation (fma((x - mean) * invstd, g, b),
    tests/_kinks._bn_z), bounded like tests/_kinks.py: at most
    max(8, 2e-4 * numel) elements may sit on a different side of a kink than
    in float64, each within 1e-5 of it.  Why: in the
    (16, 3, 2, (2, 8201, 40), hswish) case one element of channel 10 has
    z = 3.0000000215 in float64 and 2.9999998 in fp32; Hardswish's derivative
    jumps from 1.5 to 1 at z = 3, and that single flip alone moves dx by
    1.597e-3 of its max (the value round 5 measured on the GPU) and
    dbeta[10] from -119.9910 to -119.9819 — reproduced on the CPU by the
    float64 reference with the fp32 mask, no kernel involved."""
    from jabd_amd import train as T
    from _kinks import _bn_z, _region, _kink_dist, _FAMILY
    monkeypatch.setattr(T, "DGBN_RECOMPUTE", recompute)
    B, H, W = bhw
    g = torch.Generator().manual_seed(c + k * 10 + s)
    x_bn = torch.randn(B, H, W, c, generator=g) * 2 + 0.5
    gamma = 1 + 0.3 * torch.randn(c, generator=g)
    beta = 0.2 * torch.randn(c, generator=g)
    w = torch.randn(c, 1, k, k, generator=g) / k
    OH = (H + 2 * (k // 2) - k) // s + 1
    OW = (W + 2 * (k // 2) - k) // s + 1
    dy = torch.randn(B, OH, OW, c, generator=g)
    dev = torch.device(cuda)
    bn = torch.nn.BatchNorm2d(c).to(dev)
    with torch.no_grad():
        bn.weight.copy_(gamma)
        bn.bias.copy_(beta)
    xg = x_bn.to(dev)
    e_g, st = T._bn_fwd(xg, bn, act)
    wt = T.F.transpose(w.to(dev).reshape(c, k * k))
    dyg = dy.to(dev)
    dx1, dg1, db1, dw1 = T._dw_bn_bwd(dyg, e_g, wt, k, s, xg, st, act)
    de, dw2 = T._dw_bwd(dyg, e_g, wt, k, s)
    dx2, dg2, db2, _ = T._bn_bwd(de, xg, st, act)
    torch.cuda.synchronize()
    assert torch.equal(dw1, dw2)
    for a, b in ((dx1, dx2), (dg1, dg2), (db1, db2)):
        assert rel_err(a.cpu(), b.cpu()) < 1e-5
    # float64 reference: e = act(bn(x_bn)) (batch statistics), d = dwconv(e),
    # the activation's region from the HIP pre-activation
    zh = _nchw(_bn_z(x_bn, st[2], st[3], gamma, beta, None)).double()
    xr = _nchw(x_bn).double().requires_grad_()
    gr, br = gamma.double().requires_grad_(), beta.double().requires_grad_()
    z = tF.batch_norm(xr, None, None, gr, br, True, 0.0, 1e-5)
    fam = _FAMILY[act]
    flips = _region(fam, zh) != _region(fam, z.detach())
    nflip = int(flips.sum())
    assert nflip <= max(8, 2e-4 * flips.numel()), nflip
    if nflip:
        assert float(_kink_dist(fam, z.detach()[flips]).max()) < 1e-5
    e = _act_masked(z, zh, act)
    d = tF.conv2d(e, w.double(), None, s, k // 2, 1, c)
    d.backward(_nchw(dy).double())
    _check([_nchw(dx1.cpu()), dg1.cpu(), db1.cpu()], [xr.grad, gr.grad, br.grad],
           ["dx", "dgamma", "dbeta"])


@pytest.mark.gpu
@pytest.mark.parametrize("c,k,s,bhw,scale", [(72, 3, 1, (4, 40, 36), 1.0), (120, 5, 1, (3, 17, 29), 50.0),
                                             (240, 3, 2, (2, 30, 34), 1.0), (672, 5, 2, (3, 16, 16), 50.0)])
def test_dw_fwd_bn_stats(cuda, c, k, s, bhw, scale):
    """bn2's batch statistics taken by the depthwise forward kernel
    (jabd_dwconv_stats_f32 + jabd_bn_stats_final_f32) against the separate
    statistics pass (jabd_bn_stats_f32): the conv output bit-identical, mean,
    invstd and the running buffers within fp32 reassociation, including x50
    inputs whose mean dwarfs their spread (the shifted sums must not cancel)."""
    from jabd_amd import train as T
    B, H, W = bhw
    g = torch.Generator().manual_seed(c + k + s)
    x = (torch.randn(B, H, W, c, generator=g) + 3.0) * scale
    w = torch.randn(c, 1, k, k, generator=g) / k
    dev = torch.device(cuda)
    bns = []
    for _ in range(2):
        bn = torch.nn.BatchNorm2d(c).to(dev)
        with torch.no_grad():
            bn.running_mean.copy_(torch.linspace(-1, 1, c))
            bn.running_var.copy_(torch.linspace(0.5, 2, c))
        bns.append(bn)
    xg, wg = x.to(dev), w.to(dev)
    y1, _, (m1, i1) = T._dw_fwd_bn_stats(xg, wg, s, bns[0])
    y2, _ = T._dw_fwd(xg, wg, s)
    _, (_, _, m2, i2) = T._bn_fwd(y2, bns[1], "none")
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    assert rel_err(m1.cpu(), m2.cpu()) < 1e-6
    assert rel_err(i1.cpu(), i2.cpu()) < 1e-5
    assert rel_err(bns[0].running_mean.cpu(), bns[1].running_mean.cpu()) < 1e-6
    assert rel_err(bns[0].running_var.cpu(), bns[1].running_var.cpu()) < 1e-5
    ref = y2.double()
    var = ref.var((0, 1, 2), unbiased=False)
    assert rel_err(i1.cpu(), (var + bns[0].eps).rsqrt().cpu()) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,bhw,scale", [(16, 16, (4, 64, 64), 1.0), (16, 64, (2, 128, 96), 1.0),
                                                (24, 72, (3, 33, 47), 50.0), (40, 80, (2, 20, 20), 1.0),
                                                (20, 36, (1, 7, 9), 50.0), (64, 48, (2, 16, 16), 1.0),
                                                (40, 120, (2, 20, 20), 1.0)])
def test_conv1x1_bn_stats(cuda, cin, cout, bhw, scale):
    """bn1's batch statistics taken by conv1's streaming 1x1 kernel
    (jabd_conv1x1_bn_stats_f32 + jabd_bn_stats_final_f32) against the
    separate statistics pass: the conv output bit-identical to the plain
    entry point, mean / invstd / running buffers within fp32 reassociation,
    incl. x50 inputs with a large mean (shifted sums must not cancel) and a
    ragged last 16-pixel block.  Layers the streaming form does not serve
    (Cout > 80) take the 32x32 GEMM's statistics form."""
    from jabd_amd import train as T
    B, H, W = bhw
    g = torch.Generator().manual_seed(cin * cout)
    x = (torch.randn(B, H, W, cin, generator=g) + 2.0) * scale
    w = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5
    dev = torch.device(cuda)
    bns = []
    for _ in range(2):
        bn = torch.nn.BatchNorm2d(cout).to(dev)
        with torch.no_grad():
            bn.running_mean.copy_(torch.linspace(-1, 1, cout))
            bn.running_var.copy_(torch.linspace(0.5, 2, cout))
        bns.append(bn)
    xg, wg = x.to(dev), w.to(dev)
    y1, st = T._conv_fwd_bn_stats(xg, wg, bns[0])
    y2 = T._conv_fwd(xg, wg)
    torch.cuda.synchronize()
    if cout > 80:   # the 32x32 GEMM's statistics form instead (test_conv_bn_stats32)
        assert rel_err(y1.cpu(), y2.cpu()) < 1e-5
    else:
        assert torch.equal(y1, y2)
    assert st is not None, "a statistics form expected to serve this layer"
    m1, i1 = st
    _, (_, _, m2, i2) = T._bn_fwd(y2, bns[1], "none")
    torch.cuda.synchronize()
    assert rel_err(m1.cpu(), m2.cpu()) < 1e-6
    assert rel_err(i1.cpu(), i2.cpu()) < 1e-5
    assert rel_err(bns[0].running_mean.cpu(), bns[1].running_mean.cpu()) < 1e-6
    assert rel_err(bns[0].running_var.cpu(), bns[1].running_var.cpu()) < 1e-5
    ref = y2.double()
    assert rel_err(m1.cpu().double(), ref.mean((0, 1, 2)).cpu()) < 1e-6
    var = ref.var((0, 1, 2), unbiased=False)
    assert rel_err(i1.cpu(), (var + bns[0].eps).rsqrt().cpu()) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,k,stride,bhw,scale", [
    (64, 256, 1, 1, (2, 40, 36), 1.0), (256, 64, 1, 1, (3, 17, 19), 50.0),
    (64, 64, 3, 1, (2, 33, 31), 1.0), (128, 128, 3, 2, (2, 33, 31), 50.0),
    (256, 512, 1, 2, (2, 21, 18), 1.0), (512, 128, 1, 1, (1, 5, 7), 1.0),
    (16, 64, 3, 1, (2, 9, 9), 1.0)])
def test_conv_bn_stats32(cuda, cin, cout, k, stride, bhw, scale):
    """The ResNet-50 bottleneck convs' BatchNorm statistics taken in the
    32x32 GEMM's epilogue (jabd_conv_bn_stats_f32: per-32-pixel-tile mean /
    M2 rows, fp64 fixed-order combination) against an fp64 two-pass mean /
    variance of the same output and against the separate statistics pass
    (running buffers), incl. x50 inputs with a large mean, ragged last tiles
    and the stride-2 k x k / 1x1 forms.  Cin = 16 under a 3x3 kernel is not
    served: (y, None)."""
    from jabd_amd import train as T
    B, H, W = bhw
    pad = k // 2
    g = torch.Generator().manual_seed(cin * cout + k)
    x = (torch.randn(B, H, W, cin, generator=g) + 2.0) * scale
    w = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    dev = torch.device(cuda)
    bns = []
    for _ in range(2):
        bn = torch.nn.BatchNorm2d(cout).to(dev)
        with torch.no_grad():
            bn.running_mean.copy_(torch.linspace(-1, 1, cout))
            bn.running_var.copy_(torch.linspace(0.5, 2, cout))
        bns.append(bn)
    xg, wg = x.to(dev), w.to(dev)
    y1, st = T._conv_fwd_stats(xg, wg, bns[0], stride, pad)
    y2 = T._conv_fwd(xg, wg, None, stride, pad)
    torch.cuda.synchronize()
    assert y1.shape == y2.shape
    assert rel_err(y1.cpu(), y2.cpu()) < 1e-5
    if cin % 32:
        assert st is None
        return
    assert st is not None, "32x32 statistics form expected to serve this layer"
    m1, i1 = st
    _, (_, _, m2, i2) = T._bn_fwd(y1, bns[1], "none")
    torch.cuda.synchronize()
    ref = y1.double()
    mu64 = ref.mean((0, 1, 2))
    var64 = ref.var((0, 1, 2), unbiased=False)
    assert float(((m1.double() - mu64).abs() / (mu64 ** 2 + var64).sqrt()).max()) < 1e-6
    var = i1.double() ** -2 - bns[0].eps
    assert float(((var - var64).abs() / (var64 + bns[0].eps)).max()) < 1e-5
    assert rel_err(m1.cpu(), m2.cpu()) < 1e-6
    assert rel_err(i1.cpu(), i2.cpu()) < 1e-5
    assert rel_err(bns[0].running_mean.cpu(), bns[1].running_mean.cpu()) < 1e-6
    assert rel_err(bns[0].running_var.cpu(), bns[1].running_var.cpu()) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,bhw", [
    (64, 256, (2, 40, 36)), (64, 64, (3, 17, 19)), (128, 512, (2, 21, 18)), (64, 96, (1, 9, 7)),
    (128, 128, (2, 33, 31)), (64, 32, (1, 5, 3)), (128, 256, (1, 1, 1))])
def test_conv1x1_stream32_forms(cuda, cin, cout, bhw):
    """The streaming 1x1 GEMM (conv32.hip conv1x1_m32s_kernel: K = 64 / 128,
    weights resident in LDS, persistent waves over 32-pixel tiles; at K = 128
    only the plain form, the others on the tile kernel) in each of its
    epilogue forms against float64 torch: plain (no terms), bias + ReLU
    (run-time epilogue), a data gradient with the residual, the BatchNorm
    statistics form and the BatchNorm-backward sums form; ragged last tiles,
    one pixel, and N not a multiple of 128 (TN 1-3)."""
    from jabd_amd import train as T
    B, H, W = bhw
    g = torch.Generator().manual_seed(cin * 7 + cout)
    x = (torch.randn(B, H, W, cin, generator=g) + 1.0) * 3.0
    w = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5
    b = torch.randn(cout, generator=g)
    r = torch.randn(B, H, W, cout, generator=g)
    dev = torch.device(cuda)
    xg, wg, bg, rg = x.to(dev), w.to(dev), b.to(dev), r.to(dev)
    ref = x.double().reshape(-1, cin) @ w.double().reshape(cout, cin).t()
    ref = ref.reshape(B, H, W, cout)
    y0 = T._conv_fwd(xg, wg, None, 1, 0)
    pk = T._packed(wg, transposed=False)
    a = T._conv_args(xg, pk, torch.empty(B, H, W, cout, device=dev), 1, 0)
    a.bias, a.act = bg.data_ptr(), T.ACT["relu"]   # bias + ReLU: the run-time epilogue
    yb = torch.empty(B, H, W, cout, device=dev)
    a.y = yb.data_ptr()
    T.call("jabd_conv2d_nhwc_f32", T.ctypes.byref(a), T._st())
    bn = torch.nn.BatchNorm2d(cout).to(dev)
    ys, st = T._conv_fwd_stats(xg, wg, bn, 1, 0)
    # data gradient cout <- cin with the residual (the R50 conv1 data gradient's form)
    wt = w.reshape(cout, cin).t().contiguous().reshape(cin, cout, 1, 1).to(dev)
    dy = torch.randn(B, H, W, cin, generator=g)
    dres = T._dgrad_1x1_res(dy.to(dev), wt, rg)
    torch.cuda.synchronize()
    tol = 1e-5
    assert rel_err(y0.cpu().double(), ref) < tol
    assert rel_err(yb.cpu().double(), (ref + b.double()).clamp_min(0)) < tol
    assert rel_err(ys.cpu().double(), ref) < tol
    assert st is not None
    y64 = ys.cpu().double()   # the statistics of the output the kernel wrote
    mu64, var64 = y64.mean((0, 1, 2)), y64.var((0, 1, 2), unbiased=False)
    assert float(((st[0].cpu().double() - mu64).abs() / (mu64 ** 2 + var64).sqrt()).max()) < 1e-6
    var = st[1].cpu().double() ** -2 - bn.eps
    assert float(((var - var64).abs() / (var64 + bn.eps)).max()) < 1e-5
    dref = (dy.double().reshape(-1, cin) @ w.double().reshape(cout, cin).t()).reshape(B, H, W, cout)
    assert rel_err(dres.cpu().double(), dref + r.double()) < tol
    # BatchNorm-backward sums form: the data gradient is the dy of a BN + ReLU over cout
    xb = (torch.randn(B, H, W, cout, generator=g) + 0.5).to(dev)
    xm = xb.reshape(-1, cout).double()
    stb = ((1 + 0.3 * torch.randn(cout, generator=g)).to(dev),
           (0.2 * torch.randn(cout, generator=g)).to(dev),
           xm.mean(0).float(), (xm.var(0, unbiased=False) + 1e-5).rsqrt().float())
    d1, part = T._dgrad_bn_sums(dy.to(dev), wt, 1, 0, H, W, xb, stb, "relu")
    assert part is not None
    r1 = T._bn_bwd_rows(d1, xb, stb, "relu", part)
    r2 = T._bn_bwd(d1, xb, stb, "relu")
    torch.cuda.synchronize()
    assert rel_err(d1.cpu().double(), dref) < tol
    for a1, a2, name in zip(r1[:3], r2[:3], ("dx", "dgamma", "dbeta")):
        assert rel_err(a1.cpu(), a2.cpu()) < 1e-5, name


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,k,stride,bhw,scale", [
    (64, 256, 1, 1, (2, 40, 36), 1.0), (128, 512, 1, 1, (3, 17, 19), 50.0),
    (64, 64, 3, 1, (2, 33, 31), 1.0), (128, 128, 3, 1, (1, 9, 7), 50.0),
    (128, 128, 3, 2, (2, 34, 30), 1.0)])
def test_dgrad_bn_bwd_sums(cuda, cin, cout, k, stride, bhw, scale):
    """The R50 bn1 / bn2 backward sums taken in the data-gradient GEMM's
    epilogue (jabd_conv_bn_bwd_sums_f32 + jabd_bn_act_bwd_rows_f32) against
    the plain data gradient + jabd_bn_act_bwd_ex_f32 (its own reduction pass):
    the data gradient, dx, dgamma and dbeta within fp32 reassociation, incl.
    x50 inputs with a large mean and ragged tiles; a stride-2 transposed conv
    is not served (part None)."""
    from jabd_amd import train as T
    B, H, W = bhw
    pad = k // 2
    OH, OW = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    g = torch.Generator().manual_seed(cin + 7 * cout + k)
    dev = torch.device(cuda)
    w = (torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5).to(dev)
    dy = torch.randn(B, OH, OW, cout, generator=g).to(dev)
    x = ((torch.randn(B, H, W, cin, generator=g) + 2.0) * scale).to(dev)   # the BN's input
    xm = x.reshape(-1, cin).double()
    mean = xm.mean(0).float()
    invstd = (xm.var(0, unbiased=False) + 1e-5).rsqrt().float()
    gam = (1 + 0.3 * torch.randn(cin, generator=g)).to(dev)
    bet = (0.2 * torch.randn(cin, generator=g)).to(dev)
    st = (gam, bet, mean, invstd)
    d1, part = T._dgrad_bn_sums(dy, w, stride, pad, H, W, x, st, "relu")
    d2 = T._dgrad(dy, w, stride, pad, H, W)
    torch.cuda.synchronize()
    assert rel_err(d1.cpu(), d2.cpu()) < 1e-5
    if stride == 2:
        assert part is None
        return
    assert part is not None, "the BatchNorm-backward form expected to serve this conv"
    r1 = T._bn_bwd_rows(d1, x, st, "relu", part)
    r2 = T._bn_bwd(d1, x, st, "relu")
    torch.cuda.synchronize()
    for a, b, name in zip(r1[:3], r2[:3], ("dx", "dgamma", "dbeta")):
        assert rel_err(a.cpu(), b.cpu()) < 1e-5, name


@pytest.mark.gpu
@pytest.mark.parametrize("n_in,n,off", [(1, 4096, 0), (2, 1000, 0), (3, 123457 * 4, 0), (4, 64, 0),
                                        (5, 4000, 0), (2, 4001, 0), (3, 4096, 1)])
def test_sum_multi_bit_exact(cuda, n_in, n, off):
    """jabd_sum_multi_f32 (the gradient of a tensor consumed n_in times) adds
    the inputs in order — bit-identical to ((a + b) + c) + ... in torch,
    incl. inputs off 16-byte alignment."""
    import ctypes
    from jabd_amd._lib import call
    g = torch.Generator().manual_seed(n_in * 7 + n)
    xs = [torch.randn(n + off, generator=g).to(cuda)[off:] for _ in range(n_in)]
    out = torch.empty(n, device=cuda)
    ptrs = (ctypes.c_void_p * n_in)(*[x.data_ptr() for x in xs])
    call("jabd_sum_multi_f32", n_in, ptrs, n, out.data_ptr(),
         ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    ref = xs[0].clone()
    for x in xs[1:]:
        ref = ref + x
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("c,k,s,bhw,act", [(64, 3, 2, (2, 66, 50), "relu"), (72, 3, 1, (3, 31, 29), "relu"),
                                           (120, 5, 1, (2, 17, 19), "hswish"),
                                           (240, 5, 2, (2, 21, 16), "hswish")])
def test_dw_bnin(cuda, c, k, s, bhw, act):
    """Depthwise forward and weight gradient with bn1 + act applied on load
    from the pre-BN tensor (jabd_dwconv_bnin_stats_f32 /
    jabd_dw_wgrad_bnin_f32) against the same kernels on the materialised
    act(bn(x)) (jabd_bn_act_fwd_f32): outputs and statistics within fp32
    rounding of the BN expression, padding applied to the activated input."""
    from jabd_amd import train as T
    B, H, W = bhw
    g = torch.Generator().manual_seed(c * k + s)
    x = torch.randn(B, H, W, c, generator=g) * 2.0 + 0.5
    w = torch.randn(c, 1, k, k, generator=g) / k
    dev = torch.device(cuda)
    bn1 = torch.nn.BatchNorm2d(c).to(dev)
    with torch.no_grad():
        bn1.weight.copy_(torch.rand(c, generator=g) + 0.5)
        bn1.bias.copy_(torch.randn(c, generator=g) * 0.3)
    bn2s = [torch.nn.BatchNorm2d(c).to(dev) for _ in range(2)]
    xg, wg = x.to(dev), w.to(dev)
    e, st1 = T._bn_fwd(xg, bn1, act)
    y1, _, (m1, i1) = T._dw_fwd_bn_stats(xg, wg, s, bn2s[0], bnin=(st1, act))
    y2, wt, (m2, i2) = T._dw_fwd_bn_stats(e, wg, s, bn2s[1])
    torch.cuda.synchronize()
    # the on-load z is bn_act_fwd's fma((x - mean) * invstd, gamma, beta);
    # ReLU is then bit-identical, the two Hardswish formulas a few ulp apart
    if act == "relu":
        assert torch.equal(y1, y2)
    assert rel_err(y1.cpu(), y2.cpu()) < 2e-6
    assert rel_err(m1.cpu(), m2.cpu()) < 1e-5
    assert rel_err(i1.cpu(), i2.cpu()) < 1e-5
    dy = torch.randn(y2.shape, generator=g).to(dev)
    _, dw1 = T._dw_bwd(dy, xg, wt, k, s, want_dx=False, bnin=(st1, act))
    _, dw2 = T._dw_bwd(dy, e, wt, k, s, want_dx=False)
    torch.cuda.synchronize()
    if act == "relu":
        assert torch.equal(dw1, dw2)
    assert rel_err(dw1.cpu(), dw2.cpu()) < 2e-6
    # plain fp32 reference of the whole chain
    ref_e = torch.nn.functional.relu(
        torch.nn.functional.batch_norm(x.permute(0, 3, 1, 2), None, None, bn1.weight.detach().cpu(),
                                       bn1.bias.detach().cpu(), True, 0.0, bn1.eps)) \
        if act == "relu" else torch.nn.functional.hardswish(
        torch.nn.functional.batch_norm(x.permute(0, 3, 1, 2), None, None, bn1.weight.detach().cpu(),
                                       bn1.bias.detach().cpu(), True, 0.0, bn1.eps))
    ref_y = torch.nn.functional.conv2d(ref_e, w, None, s, k // 2, 1, c)
    assert rel_err(y1.cpu().permute(0, 3, 1, 2), ref_y) < 1e-4


def _near_kink_bn(C=64, n=16, seed=21):
    """Per channel a BN (mean, invstd, gamma, beta) and n consecutive fp32
    inputs straddling the point where z = (x - mean) * invstd * gamma + beta
    crosses 0 (the ReLU kink), as numpy float32."""
    import numpy as np
    r = np.random.default_rng(seed)
    mu = r.uniform(-1, 1, C).astype(np.float32)
    inv = r.uniform(0.3, 3.0, C).astype(np.float32)
    gam = (r.uniform(0.4, 1.6, C) * r.choice([-1, 1], C)).astype(np.float32)
    bet = r.uniform(-0.6, 0.6, C).astype(np.float32)
    x0 = (mu.astype(np.float64) - bet.astype(np.float64) / (inv.astype(np.float64) * gam)).astype(np.float32)
    xs = np.empty((n, C), np.float32)
    for c in range(C):
        v = x0[c]
        for _ in range(n // 2):
            v = np.nextafter(v, np.float32(-np.inf))
        for i in range(n):
            xs[i, c] = v
            v = np.nextafter(v, np.float32(np.inf))
    return mu, inv, gam, bet, xs


def _fma32_np(a, b, c):
    import numpy as np
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(np.float32)


def test_near_kink_inputs_separate_the_bn_forms():
    """The inputs of test_dw_bnin_kink_masks are sensitive: the folded
    on-load form fma(x, invstd * gamma, beta - mean * invstd * gamma) and
    the BN kernels' fma((x - mean) * invstd, gamma, beta) put some of them on
    different sides of the ReLU kink (so a forward that used the folded form
    while the backward masks with the other would fail that test)."""
    import numpy as np
    mu, inv, gam, bet, xs = _near_kink_bn()
    a = inv * gam
    c = _fma32_np(-mu, a, bet)
    z_fold = _fma32_np(xs, a[None], c[None])
    z_bn = _fma32_np((xs - mu[None]) * inv[None], gam[None], bet[None])
    flips = int(((z_fold > 0) != (z_bn > 0)).sum())
    assert flips >= 5, flips
    # and every channel's window does cross the kink under the BN form
    assert bool(((z_bn > 0).any(0) & (z_bn <= 0).any(0)).all())


@pytest.mark.gpu
@pytest.mark.parametrize("recompute", [True, False])
def test_dw_bnin_kink_masks(cuda, recompute, monkeypatch):
    """the BN-input depthwise forward's activation region must be
    the mask its backward applies, element for element, next to the kink.
    A centre-tap-only 3x3/s2 depthwise weight makes the forward output at
    (oh, ow) = relu(z(x[2oh, 2ow])) and the input gradient reach only those
    pixels; dy = 2^j on 16 of them makes bn1's dbeta = sum_j 2^j [z_j > 0]
    an exact bit mask of the backward's region (sums of distinct powers of
    two below 2^24 are exact in fp32)."""
    import numpy as np
    from jabd_amd import train as T
    monkeypatch.setattr(T, "DGBN_RECOMPUTE", recompute)
    C, n = 64, 16
    mu, inv, gam, bet, xs = _near_kink_bn(C, n)
    H = W = 16
    x = np.empty((1, H, W, C), np.float32)
    far = (mu - np.sign(gam) * 50.0 / (inv * np.abs(gam))).astype(np.float32)   # z ~ -50
    x[:] = far
    pos = [(2 * (j // 4), 2 * (j % 4)) for j in range(n)]
    for j, (ih, iw) in enumerate(pos):
        x[0, ih, iw] = xs[j]
    dev = torch.device(cuda)
    xg = torch.from_numpy(x).to(dev)
    w = torch.zeros(C, 1, 3, 3)
    w[:, 0, 1, 1] = 1.0
    wg = w.to(dev)
    st = tuple(torch.from_numpy(t).to(dev) for t in (gam, bet, mu, inv))
    bn2 = torch.nn.BatchNorm2d(C).to(dev)
    y, wt, _ = T._dw_fwd_bn_stats(xg, wg, 2, bn2, bnin=(st, "relu"))
    dy = torch.zeros(1, 8, 8, C)
    for j, (ih, iw) in enumerate(pos):
        dy[0, ih // 2, iw // 2] = float(2 ** j)
    dx, dgamma, dbeta, dw = T._dw_bn_bwd(dy.to(dev), None, wt, 3, 2, xg, st, "relu")
    torch.cuda.synchronize()
    yc = y.cpu().numpy()
    fwd = np.stack([yc[0, ih // 2, iw // 2] > 0 for ih, iw in pos])          # [n, C]
    bits = dbeta.cpu().numpy().astype(np.int64)
    bwd = np.stack([(bits >> j) & 1 for j in range(n)]).astype(bool)
    assert (dbeta.cpu().numpy() == bits).all()
    bad = np.argwhere(fwd != bwd)
    assert bad.size == 0, f"{len(bad)} elements: forward region != backward mask, e.g. {bad[:4]}"
    # each channel's window straddles the kink, so the check is not vacuous
    assert fwd.any(0).all() and (~fwd).any(0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("bhwc", [(2, 17, 23, 64), (1, 64, 64, 8), (3, 9, 8, 12), (1, 9, 37, 256)])
def test_maxpool_idx_forms_bit_identical(cuda, bhwc):
    """The training max-pool (argmax kept as a uint8 window position) gives
    the eval max-pool's values and the recomputing backward's gradient bit for
    bit — with exact ties (quantised inputs), -inf and NaN in the windows."""
    import ctypes
    from jabd_amd import functional as F
    from jabd_amd._lib import call
    B, H, W, C = bhwc
    g = torch.Generator().manual_seed(B * H + C)
    x = torch.round(torch.randn(B, H, W, C, generator=g) * 2) / 2      # many ties
    x.view(-1)[::97] = float("-inf")
    x.view(-1)[::211] = float("nan")
    x = x.to(cuda)
    OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    y = torch.empty(B, OH, OW, C, device=cuda)
    idx = torch.empty(B, OH, OW, C, dtype=torch.uint8, device=cuda)
    call("jabd_maxpool_idx_nhwc_f32", x.data_ptr(), B, H, W, C, 3, 2, 1, y.data_ptr(),
         idx.data_ptr(), st)
    y_eval = F.maxpool(x, 3, 2, 1)
    dy = torch.randn(B, OH, OW, C, generator=g).to(cuda)
    dx1 = torch.empty_like(x)
    dx2 = torch.empty_like(x)
    call("jabd_maxpool_bwd_idx_f32", idx.data_ptr(), dy.data_ptr(), B, H, W, C, 3, 2, 1,
         dx1.data_ptr(), st)
    call("jabd_maxpool_bwd_f32", x.data_ptr(), dy.data_ptr(), B, H, W, C, 3, 2, 1,
         dx2.data_ptr(), st)
    torch.cuda.synchronize()
    assert torch.equal(y.nan_to_num(7.0), y_eval.nan_to_num(7.0))
    assert torch.equal(dx1, dx2)
    # and torch's own max_pool2d backward (first maximum, NaN propagating)
    xc = x.permute(0, 3, 1, 2).cpu().double().requires_grad_()
    yc = torch.nn.functional.max_pool2d(xc, 3, 2, 1)
    yc.backward(dy.permute(0, 3, 1, 2).cpu().double())
    assert torch.allclose(dx1.permute(0, 3, 1, 2).cpu().double(), xc.grad, rtol=1e-6, atol=1e-6)
