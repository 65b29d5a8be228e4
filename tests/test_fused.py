"""Fused MobileNetV3 expand 1x1 + depthwise kernel (csrc/expdw.hip) against
a PyTorch fp32 reference of the same folded ops (nets/mobilenetV3.py:141-142)
and against the two-kernel HIP path, for every Block_eca geometry of
JABD-MNv3 (k, stride, Cin, E) on ragged map sizes."""
import pytest
import torch
import torch.nn.functional as tF

from _util import rel_err

# (k, Cin, E, stride, act) — the 15 Block_eca specs of nets/mobilenetV3.py:452-522
BLOCKS = [(3, 16, 16, 1, "relu"), (3, 16, 64, 2, "relu"), (3, 24, 72, 1, "relu"),
          (5, 24, 72, 2, "relu"), (5, 40, 120, 1, "relu"), (3, 40, 240, 2, "hswish"),
          (3, 80, 200, 1, "hswish"), (3, 80, 184, 1, "hswish"), (3, 80, 480, 1, "hswish"),
          (3, 112, 672, 1, "hswish"), (5, 112, 672, 2, "hswish"), (5, 160, 960, 1, "hswish")]


def _act(x, act):
    return tF.relu(x) if act == "relu" else tF.hardswish(x)


@pytest.mark.gpu
@pytest.mark.parametrize("spec", BLOCKS, ids=lambda s: "k%d_c%d_e%d_s%d" % s[:4])
@pytest.mark.parametrize("hw", [(37, 29), (64, 64)])
def test_expand_dw_parity(cuda, spec, hw):
    from jabd_amd import functional as F
    k, cin, E, s, act = spec
    H, W = hw
    g = torch.Generator().manual_seed(k * 1000 + cin + E + s)
    B = 2
    x = torch.randn(B, cin, H, W, generator=g)
    conv1 = torch.nn.Conv2d(cin, E, 1, bias=False)
    bn1 = torch.nn.BatchNorm2d(E)
    conv2 = torch.nn.Conv2d(E, E, k, s, k // 2, groups=E, bias=False)
    bn2 = torch.nn.BatchNorm2d(E)
    with torch.no_grad():
        conv1.weight.copy_(torch.randn(conv1.weight.shape, generator=g) / cin ** 0.5)
        conv2.weight.copy_(torch.randn(conv2.weight.shape, generator=g) / k)
        for bn in (bn1, bn2):
            bn.weight.copy_(1 + 0.2 * torch.randn(E, generator=g))
            bn.bias.copy_(0.3 * torch.randn(E, generator=g))
            bn.running_mean.copy_(0.1 * torch.randn(E, generator=g))
            bn.running_var.copy_(0.5 + torch.rand(E, generator=g))
    for m in (conv1, bn1, conv2, bn2):
        m.eval()
    with torch.no_grad():
        ref = _act(bn2(conv2(_act(bn1(conv1(x)), act))), act)
    pk = F.pack_conv(conv1.to(cuda), bn1.to(cuda))
    dw_w, dw_b = F.pack_dw(conv2.to(cuda), bn2.to(cuda))
    xg = x.permute(0, 2, 3, 1).contiguous().to(cuda)
    y, part = F.expand_dw(xg, pk, dw_w, dw_b, k, s, act=act)
    torch.cuda.synchronize()
    got = y.permute(0, 3, 1, 2).cpu()
    assert got.shape == ref.shape
    assert rel_err(got, ref) < 2e-5, rel_err(got, ref)
    # ECA pool partials: per-image channel sums of the activated output
    sums = part.sum(1).cpu().double()
    assert rel_err(sums, ref.double().sum((2, 3))) < 1e-5
    if s == 2:  # the block's dw3x3/s2 + BN skip branch fused on the same input tile
        sdw = torch.nn.Conv2d(cin, cin, 3, 2, 1, groups=cin, bias=False)
        sbn = torch.nn.BatchNorm2d(cin)
        with torch.no_grad():
            sdw.weight.copy_(torch.randn(sdw.weight.shape, generator=g) / 3)
            sbn.weight.copy_(1 + 0.2 * torch.randn(cin, generator=g))
            sbn.bias.copy_(0.3 * torch.randn(cin, generator=g))
            sbn.running_mean.copy_(0.1 * torch.randn(cin, generator=g))
            sbn.running_var.copy_(0.5 + torch.rand(cin, generator=g))
            sref = sbn.eval()(sdw(x))
        skw, skb = F.pack_dw(sdw.to(cuda), sbn.to(cuda))
        y3, part3, t = F.expand_dw(xg, pk, dw_w, dw_b, k, s, act=act, skip=(skw, skb))
        assert torch.equal(y3, y)
        assert rel_err(t.permute(0, 3, 1, 2).cpu(), sref) < 2e-5
        t2, _ = F.dwconv(xg, skw, skb, 3, 2)
        assert rel_err(t, t2) < 2e-6
    # the two-kernel path computes the same tensor
    e = F.conv(xg, pk, act=act)
    y2, part2 = F.dwconv(e, dw_w, dw_b, k, s, act=act, partials=True)
    assert rel_err(y, y2) < 2e-5


@pytest.mark.gpu
@pytest.mark.parametrize("act", ["hswish", "relu", "none"])
@pytest.mark.parametrize("hw", [(37, 29), (128, 96), (1, 2), (17, 130), (6, 1024)])
def test_stem_parity(cuda, act, hw):
    """MNv3 stem (nets/mobilenetV3.py:455-457,511): conv3x3/s2/p1 3->16 on the
    NCHW input + folded bias + act, NHWC out, vs torch fp32 conv2d."""
    from jabd_amd import functional as F
    H, W = hw
    g = torch.Generator().manual_seed(H * 131 + W)
    x = torch.randn(3, 3, H, W, generator=g) * 50
    w = torch.randn(16, 3, 3, 3, generator=g) / 27 ** 0.5
    b = torch.randn(16, generator=g)
    ref = tF.conv2d(x, w, b, stride=2, padding=1)
    ref = {"hswish": tF.hardswish, "relu": tF.relu, "none": lambda t: t}[act](ref)
    wp = w.permute(2, 3, 1, 0).reshape(27, 16).contiguous()  # [(kh,kw,ci)][co]
    y = F.stem(x.to(cuda), wp.to(cuda), b.to(cuda), act)
    torch.cuda.synchronize()
    got = y.permute(0, 3, 1, 2).cpu()
    assert got.shape == ref.shape
    assert rel_err(got, ref) < 2e-6, rel_err(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,split,hw,gate", [(40, 40, 0, (128, 96), False),
                                                     (40, 32, 20, (37, 29), True),
                                                     (12, 24, 12, (23, 50), False),
                                                     (64, 48, 0, (9, 17), True),
                                                     (12, 12, 0, (3, 5), False)])
def test_conv3x3_tile_parity(cuda, cin, cout, split, hw, gate):
    """The LDS-tiled 3x3 / stride-1 kernel (conv3x3_tile_kernel: SSH branches,
    FPN merges) vs torch fp32 conv2d: ragged tiles, the ECA gate applied while
    staging, and the split output of the fused SSH branches."""
    from jabd_amd import functional as F
    H, W = hw
    g = torch.Generator().manual_seed(cin * 7 + cout + H)
    B = 2
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / (9 * cin) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    sc = torch.rand(B, cin, generator=g) if gate else None
    xin = x * sc[:, :, None, None] if gate else x
    ref = tF.conv2d(xin, w, b, padding=1)
    conv = torch.nn.Conv2d(cin, cout, 3, padding=1)
    with torch.no_grad():
        conv.weight.copy_(w)
        conv.bias.copy_(b)
    pk = F.pack_conv(conv.to(cuda))
    xg = x.permute(0, 2, 3, 1).contiguous().to(cuda)
    asc = sc.to(cuda).contiguous() if gate else None
    if split:
        y = torch.empty((B, H, W, split), device=cuda)
        y2 = torch.empty((B, H, W, cout - split), device=cuda)
        F.conv(xg, pk, pad=1, act="relu", ascale=asc, out=y, y2=y2, nsplit=split,
               act2="leaky", slope2=0.1)
        got = torch.cat([y, y2], -1).permute(0, 3, 1, 2).cpu()
        want = torch.cat([tF.relu(ref[:, :split]), tF.leaky_relu(ref[:, split:], 0.1)], 1)
    else:
        got = F.conv(xg, pk, pad=1, act="relu", ascale=asc).permute(0, 3, 1, 2).cpu()
        want = tF.relu(ref)
    assert rel_err(got, want) < 2e-5, rel_err(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cin2,cout,gate,res,hw,act", [
    (16, 0, 16, True, True, (33, 31), "relu"),      # KC 1, ragged last block
    (64, 16, 24, True, False, (17, 23), "relu"),    # K-concat skip source (b2)
    (72, 0, 24, True, True, (16, 16), "relu"),      # KC 5 with a half stage (b3)
    (120, 0, 40, True, True, (8, 40), "hswish"),    # KC 8, TN 3 (b5)
    (40, 0, 40, False, False, (31, 7), "leaky"),    # FPN lateral
    (200, 0, 80, True, True, (12, 13), "hswish"),   # 8-wave workgroups (b8)
    (240, 40, 80, True, False, (5, 9), "hswish"),   # KC 18 + K-concat (b7)
])
def test_conv1x1_stream_parity(cuda, cin, cin2, cout, gate, res, hw, act):
    """The streaming 1x1 kernel (conv_stream.hip: persistent workgroups, LDS
    weights + gates, next block's K stages in flight) vs torch fp32: ragged
    pixel counts, half-filled K stages, the K-concatenated skip source, the
    ECA gate on the first source only, residual and activation."""
    from jabd_amd import functional as F
    H, W = hw
    B = 3
    g = torch.Generator().manual_seed(cin * 5 + cout + H)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    sc = torch.rand(B, cin, generator=g) if gate else None
    ref = tF.conv2d(x * sc[:, :, None, None] if gate else x, w, b)
    extra = None
    if cin2:
        x2 = torch.randn(B, cin2, H, W, generator=g)
        w2 = torch.randn(cout, cin2, generator=g) / cin2 ** 0.5
        t2 = torch.randn(cout, generator=g) * 0.1
        ref = ref + tF.conv2d(x2, w2[:, :, None, None], t2)
        extra = (w2.t().contiguous().to(cuda), t2.to(cuda))
    r = torch.randn(B, cout, H, W, generator=g) if res else None
    if res:
        ref = ref + r
    want = {"relu": tF.relu, "hswish": tF.hardswish,
            "leaky": lambda v: tF.leaky_relu(v, 0.1)}[act](ref)
    conv = torch.nn.Conv2d(cin, cout, 1)
    with torch.no_grad():
        conv.weight.copy_(w)
        conv.bias.copy_(b)
    pk = F.pack_conv(conv.to(cuda), extra=extra)
    nhwc = lambda v: v.permute(0, 2, 3, 1).contiguous().to(cuda)  # noqa: E731
    y = F.conv(nhwc(x), pk, act=act, slope=0.1, ascale=sc.to(cuda).contiguous() if gate else None,
               x2=nhwc(x2) if cin2 else None, res=nhwc(r) if res else None)
    got = y.permute(0, 3, 1, 2).cpu()
    assert rel_err(got, want) < 2e-5, rel_err(got, want)


@pytest.mark.gpu
def test_eca_gates_multi_equal_per_tensor(cuda):
    """The head's three ECA gates in one pool + gate launch pair
    (jabd_eca_pool_gate_multi_f32) equal the per-tensor pool + gate, bit for
    bit, on the pyramid shapes (40/80/160 channels, 32/16/8 maps) and on a
    channel-offset view (pixel stride > C)."""
    from jabd_amd import functional as F
    g = torch.Generator().manual_seed(5)
    xs = [torch.randn(3, s, s, c, generator=g).to(cuda) for s, c in ((32, 40), (16, 80), (8, 160))]
    wide = torch.randn(3, 12, 12, 48, generator=g).to(cuda)
    xs.append(wide[..., 8:48])  # 40 channels at pixel stride 48
    ws = [torch.randn(k, generator=g).to(cuda) for k in (3, 3, 5, 3)]
    got = F.eca_gates_multi(xs, ws, "sigmoid")
    assert got is not None
    for x, w, s in zip(xs, ws, got):
        xc = x.contiguous()
        ref = F.eca_gate(F.channel_sums(xc), xc.shape[1] * xc.shape[2], w, "sigmoid")
        assert torch.equal(s, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("spec", BLOCKS + [(3, 24, 72, 1, "none")],
                         ids=lambda s: "k%d_c%d_e%d_s%d_%s" % s)
@pytest.mark.parametrize("bhw", [(4, 96, 80), (3, 37, 29), (1, 1, 2)])
def test_expand_dw_forms_bit_identical(cuda, spec, bhw):
    """The wave-specialised persistent kernel (expand waves feeding
    double-buffered tiles to depthwise waves), the persistent per-chunk kernel
    (expdw2.hip, opt-in) and the one-item-per-workgroup kernel (the default) compute
    every output with the same operation sequence: y, the ECA partials and
    the fused skip branch must be bit-identical.  (4, 96, 80)
    gives several items per persistent workgroup (the expanded-buffer and
    tap/partial rings wrap), (1, 1, 2) a grid smaller than the CU count.

    Exception (round 6): for Cin 24 (two input stages) the default kernel
    runs the 8-channel last input stage as 2 MFMAs over channels 4e + g
    instead of 4 over channels 4g + e (csrc/expdw.hip, tail8), so its k sum
    is taken in another order: there forms 2 / 3 / 4 stay bit-identical to
    each other, form 1 agrees with them within 1e-6 and its skip branch
    (no MFMA) bit for bit."""
    from jabd_amd import functional as F
    from jabd_amd._lib import lib
    k, cin, E, s, act = spec
    B, H, W = bhw
    g = torch.Generator().manual_seed(k * 7 + cin + E + H)
    conv1 = torch.nn.Conv2d(cin, E, 1)
    conv2 = torch.nn.Conv2d(E, E, k, s, k // 2, groups=E)
    sdw = torch.nn.Conv2d(cin, cin, 3, 2, 1, groups=cin)
    with torch.no_grad():
        for c in (conv1, conv2, sdw):
            c.weight.copy_(torch.randn(c.weight.shape, generator=g) / c.weight[0].numel() ** 0.5)
            c.bias.copy_(0.3 * torch.randn(c.bias.shape, generator=g))
    pk = F.pack_conv(conv1.to(cuda))
    tapmajor = lambda c: (c.weight.detach().reshape(c.weight.shape[0], -1).t().contiguous().to(cuda),  # noqa: E731
                          c.bias.detach().contiguous().to(cuda))
    dw_w, dw_b = tapmajor(conv2)
    skw, skb = tapmajor(sdw)
    x = torch.randn(B, H, W, cin, generator=g).to(cuda)
    outs = []
    try:
        for form in (1, 2, 3):
            lib().jabd_expand_dw_select(form)
            if s == 2:
                outs.append(F.expand_dw(x, pk, dw_w, dw_b, k, s, act=act, skip=(skw, skb)))
            else:
                outs.append(F.expand_dw(x, pk, dw_w, dw_b, k, s, act=act))
    finally:
        lib().jabd_expand_dw_select(0)
    torch.cuda.synchronize()
    tail8 = cin == 24
    for a, b in zip(outs[1], outs[2]):
        assert torch.equal(a, b)
    for i, (a, b) in enumerate(zip(outs[0], outs[1])):
        if tail8 and i < 2:
            assert rel_err(a, b) < 1e-6, rel_err(a, b)
        else:
            assert torch.equal(a, b)
    # the chunk-pipelined form (4, csrc/expdw3.hip; opt-in: JABD_EXPDW3=1
    # or select(4), measured slower than expdw1): y and the skip branch bit-identical, the ECA partials (a sum
    # over the tile in another fixed order) within 2e-6 relative
    try:
        lib().jabd_expand_dw_select(4)
        if s == 2:
            o4 = F.expand_dw(x, pk, dw_w, dw_b, k, s, act=act, skip=(skw, skb))
        else:
            o4 = F.expand_dw(x, pk, dw_w, dw_b, k, s, act=act)
    finally:
        lib().jabd_expand_dw_select(0)
    torch.cuda.synchronize()
    assert torch.equal(o4[0], outs[1][0])
    if s == 2:
        assert torch.equal(o4[2], outs[1][2])
    assert rel_err(o4[1], outs[1][1]) < 2e-6


@pytest.mark.gpu
@pytest.mark.parametrize("spec", [BLOCKS[1], BLOCKS[2], BLOCKS[5]],
                         ids=lambda s: "k%d_c%d_e%d_s%d" % s[:4])
def test_expand_dw_nan_rule(cuda, spec):
    """NaN inputs: the fused expand+depthwise kernel, the two-kernel path and
    PyTorch put NaN at the same outputs (every ReLU keeps NaN, as torch.relu;
    csrc/common.h relu_f), and agree elsewhere."""
    from jabd_amd import functional as F
    k, cin, E, s, act = spec
    g = torch.Generator().manual_seed(31)
    B, H, W = 2, 33, 40
    x = torch.randn(B, cin, H, W, generator=g)
    x[0, 3, 5, 7] = float("nan")
    x[1, :, 20, 31] = float("nan")
    conv1 = torch.nn.Conv2d(cin, E, 1, bias=False)
    conv2 = torch.nn.Conv2d(E, E, k, s, k // 2, groups=E, bias=False)
    bn1, bn2 = torch.nn.BatchNorm2d(E).eval(), torch.nn.BatchNorm2d(E).eval()
    with torch.no_grad():
        conv1.weight.copy_(torch.randn(conv1.weight.shape, generator=g) / cin ** 0.5)
        conv2.weight.copy_(torch.randn(conv2.weight.shape, generator=g) / k)
        for bn in (bn1, bn2):
            bn.bias.copy_(0.3 * torch.randn(E, generator=g))
        e_ref = _act(bn1(conv1(x)), act)
        ref = _act(bn2(conv2(e_ref)), act)
    pk = F.pack_conv(conv1.to(cuda), bn1.to(cuda))
    dw_w, dw_b = F.pack_dw(conv2.to(cuda), bn2.to(cuda))
    xg = x.permute(0, 2, 3, 1).contiguous().to(cuda)
    y, _ = F.expand_dw(xg, pk, dw_w, dw_b, k, s, act=act)
    e = F.conv(xg, pk, act=act)
    y2, _ = F.dwconv(e, dw_w, dw_b, k, s, act=act, partials=True)
    got = y.permute(0, 3, 1, 2).cpu()
    got2 = y2.permute(0, 3, 1, 2).cpu()
    nan = torch.isnan(ref)
    assert int(nan.sum()) > 0
    assert torch.equal(torch.isnan(got), nan)
    assert torch.equal(torch.isnan(got2), nan)
    assert torch.equal(torch.isnan(e.cpu()), torch.isnan(e_ref.permute(0, 2, 3, 1)))
    assert rel_err(got[~nan], ref[~nan]) < 2e-5
    assert rel_err(got2[~nan], ref[~nan]) < 2e-5


@pytest.mark.gpu
@pytest.mark.parametrize("hw", [(37, 29), (64, 64), (18, 17)])
@pytest.mark.parametrize("act", ["relu", "hswish"])
def test_expand_dw_fused_previous_project(cuda, hw, act):
    """Blocks 1 -> 2 of JABD-MNv3 (nets/mobilenetV3.py:144-150, 452-456): block
    1's project (16 -> 16 1x1 + folded BN, ECA gate, identity residual, act)
    run inside block 2's fused kernel (jabd_expdw_args.pw) against the same
    ops launched separately (F.conv, then F.expand_dw on its output): y, the
    ECA partials and the fused skip branch within fp32 reassociation (the
    project's k sum is taken in the MFMA's order instead of the streaming
    kernel's)."""
    from jabd_amd import functional as F
    H, W = hw
    B, C, E = 2, 16, 64
    g = torch.Generator().manual_seed(H * 7 + W)

    def conv_bn(cin, cout, k, s, groups=1):
        c = torch.nn.Conv2d(cin, cout, k, s, k // 2, groups=groups, bias=False)
        bn = torch.nn.BatchNorm2d(cout)
        with torch.no_grad():
            c.weight.copy_(torch.randn(c.weight.shape, generator=g) / c.weight[0].numel() ** 0.5)
            bn.weight.copy_(1 + 0.2 * torch.randn(cout, generator=g))
            bn.bias.copy_(0.3 * torch.randn(cout, generator=g))
            bn.running_mean.copy_(0.1 * torch.randn(cout, generator=g))
            bn.running_var.copy_(0.5 + torch.rand(cout, generator=g))
        return c.eval().to(cuda), bn.eval().to(cuda)

    p_conv, p_bn = conv_bn(C, C, 1, 1)
    e_conv, e_bn = conv_bn(C, E, 1, 1)
    d_conv, d_bn = conv_bn(E, E, 3, 2, groups=E)
    s_conv, s_bn = conv_bn(C, C, 3, 2, groups=C)
    pk_p = F.pack_conv(p_conv, p_bn)
    pk_e = F.pack_conv(e_conv, e_bn)
    dw_w, dw_b = F.pack_dw(d_conv, d_bn)
    skw, skb = F.pack_dw(s_conv, s_bn)
    d0 = torch.randn(B, H, W, C, generator=g).relu().to(cuda)   # block 1's depthwise output
    x0 = torch.randn(B, H, W, C, generator=g).to(cuda)          # block 1's input (residual)
    gate = torch.rand(B, C, generator=g).to(cuda)
    out0 = F.conv(d0, pk_p, act=act, ascale=gate, res=x0)
    ref = F.expand_dw(out0, pk_e, dw_w, dw_b, 3, 2, act=act, skip=(skw, skb))
    got = F.expand_dw(d0, pk_e, dw_w, dw_b, 3, 2, act=act, skip=(skw, skb),
                      pre=(pk_p, gate, x0, act))
    torch.cuda.synchronize()
    for name, a, b in zip(("y", "partials", "skip"), got, ref):
        assert rel_err(a, b) < 1e-5, (name, rel_err(a, b))


@pytest.mark.gpu
def test_engine_fused_previous_project(cuda, monkeypatch):
    """The eval plan takes the fused-project form for JABD-MNv3 blocks 1 -> 2
    (engine.FUSE_PRE) and agrees with the separate launches (FUSE_PRE off)."""
    from jabd_amd import engine, functional as F
    from test_model import _mnv3
    m = _mnv3().to(cuda).eval()
    x = torch.randn(2, 3, 160, 128, generator=torch.Generator().manual_seed(3)).to(cuda)
    calls = []
    orig = F.expand_dw

    def spy(*a, **kw):
        calls.append(kw.get("pre") is not None)
        return orig(*a, **kw)

    monkeypatch.setattr(F, "expand_dw", spy)
    with torch.no_grad():
        monkeypatch.setattr(engine, "FUSE_PRE", True)
        got = m(x)
        assert calls.count(True) == 1, calls
        monkeypatch.setattr(engine, "FUSE_PRE", False)
        calls.clear()
        ref = m(x)
        assert not any(calls)
    for a, b in zip(got, ref):
        assert rel_err(a, b) < 1e-5, rel_err(a, b)
