"""ORACLE (test infrastructure only) — PyTorch-CPU fp32 restatement of the
JABD detector forward (and, through autograd, its backward).

Functional: every function takes a flat `state_dict`-style mapping `P`
whose keys are the reference's own parameter names, so one set of weights
drives both this restatement and the product module.  Paths are relative to
/root/reference/JABD2080ti.

  * JABD-MobileNetV3  — nets/retinaface_r.py:228-343 over
    nets/mobilenetV3.py:452-522 (MobileNetV3_Large_eca, Block_eca :94-150,
    in-block eca_block :332-348 with Hardsigmoid).
  * RetinaFace-R50 + ECA + NLM — nets/retinaface_eca_nonlocal.py:235-359
    over torchvision.models.resnet50 (layout identical to
    nets/resnet_pytorch_r.py:87-303).
  * JABD-MobileNetV3-BECA — train_mobilenetV3_ecagai.py:161-435 (defined
    inline in that training script).
"""
import math

import torch
import torch.nn.functional as F

# (kernel, in, expand, out, act, se, stride) — nets/mobilenetV3.py:459-481
MNV3_LAYERS = [
    [(3, 16, 16, 16, "relu", False, 1), (3, 16, 64, 24, "relu", False, 2),
     (3, 24, 72, 24, "relu", False, 1), (5, 24, 72, 40, "relu", True, 2),
     (5, 40, 120, 40, "relu", True, 1), (5, 40, 120, 40, "relu", True, 1)],
    [(3, 40, 240, 80, "hswish", False, 2), (3, 80, 200, 80, "hswish", False, 1),
     (3, 80, 184, 80, "hswish", False, 1), (3, 80, 184, 80, "hswish", False, 1)],
    [(3, 80, 480, 112, "hswish", True, 1), (3, 112, 672, 112, "hswish", True, 1),
     (5, 112, 672, 160, "hswish", True, 2), (5, 160, 672, 160, "hswish", True, 1),
     (5, 160, 960, 160, "hswish", True, 1)],
]

R50_LAYERS = [(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]  # (width, blocks, stride)


def eca_kernel_size(channel, b=1, gamma=2):
    """nets/mobilenetV3.py:335-336 / nets/retinaface_r.py:211-212."""
    k = int(abs((math.log(channel, 2) + b) / gamma))
    return k if k % 2 else k + 1


# ----------------------------------------------------------------------------- kinks
# Every activation whose derivative jumps (ReLU, LeakyReLU, Hardswish,
# Hardsigmoid) and the max-pool argmax go through kink() / maxpool().  By
# default they are the plain torch ops.  With REPLAY set (tests/_kinks.py) a
# call asks REPLAY.match(kind, z) for the HIP forward's own pre-activation of
# the same tensor; the forward value stays this run's, and the backward takes
# the derivative's region (which side of each kink) from the HIP tensor.  An
# element within fp32 rounding of a kink then has the same mask in both runs,
# so a gradient comparison measures the kernels, not the mask flips.
REPLAY = None

_ACT_FN = {
    "relu": lambda z, s: F.relu(z),
    "leaky": lambda z, s: F.leaky_relu(z, s),
    "hswish": lambda z, s: F.hardswish(z),
    "hsigmoid": lambda z, s: F.hardsigmoid(z),
}


class _KinkFn(torch.autograd.Function):
    """act(z) whose backward uses the region of zr (PyTorch's *_backward
    conventions: relu/leaky z > 0; hardswish z < -3 -> 0, z <= 3 -> z/3 + 1/2,
    else 1; hardsigmoid 1/6 on (-3, 3))."""

    @staticmethod
    def forward(ctx, z, zr, kind, slope):
        ctx.save_for_backward(z, zr)
        ctx.cfg = (kind, slope)
        return _ACT_FN[kind](z, slope)

    @staticmethod
    def backward(ctx, g):
        z, zr = ctx.saved_tensors
        kind, slope = ctx.cfg
        one, zero = torch.ones_like(z), torch.zeros_like(z)
        if kind in ("relu", "leaky"):
            d = torch.where(zr > 0, one, zero + (slope if kind == "leaky" else 0.0))
        elif kind == "hswish":
            d = torch.where(zr < -3, zero, torch.where(zr <= 3, z / 3 + 0.5, one))
        else:
            d = torch.where((zr > -3) & (zr < 3), one / 6, zero)
        return g * d, None, None, None


def kink(z, kind, slope=0.0):
    if REPLAY is not None:
        zr = REPLAY.match(kind, z)
        if zr is not None:
            return _KinkFn.apply(z, zr.to(z.dtype), kind, slope)
    return _ACT_FN[kind](z, slope)


def maxpool(x, k=3, s=2, p=1):
    """F.max_pool2d(x, 3, 2, 1); under REPLAY the argmax of each window is the
    HIP input's (first maximum in scan order, as torch's and the kernel's)."""
    if REPLAY is not None:
        xr = REPLAY.match("maxpool", x)
        if xr is not None:
            _, idx = F.max_pool2d(xr.double(), k, s, p, return_indices=True)
            return x.flatten(2).gather(2, idx.flatten(2)).view(idx.shape)
    return F.max_pool2d(x, k, s, p)


def _act(x, kind):
    if kind in ("relu", "hswish"):
        return kink(x, kind)
    if kind is None:
        return x
    raise ValueError(kind)


class Ctx:
    """Batch-norm mode: eval (running stats) or train (batch stats + update)."""

    def __init__(self, P, train=False, momentum=0.1, eps=1e-5):
        self.P, self.train, self.momentum, self.eps = P, train, momentum, eps

    def bn(self, x, name):
        P = self.P
        return F.batch_norm(x, P[name + ".running_mean"], P[name + ".running_var"],
                            P[name + ".weight"], P[name + ".bias"], self.train, self.momentum,
                            self.eps)

    def conv(self, x, name, stride=1, padding=0, groups=1):
        b = self.P.get(name + ".bias")
        return F.conv2d(x, self.P[name + ".weight"], b, stride, padding, 1, groups)


def eca(ctx, x, name, gate):
    """ECA: global average pool -> Conv1d over channels -> gate -> x*y."""
    w = ctx.P[name + ".conv.weight"]
    k = w.shape[-1]
    y = x.mean(dim=(2, 3))                                # AdaptiveAvgPool2d(1)
    y = F.conv1d(y.unsqueeze(1), w, padding=(k - 1) // 2).squeeze(1)
    y = torch.sigmoid(y) if gate == "sigmoid" else kink(y, "hsigmoid")
    return x * y[:, :, None, None]


def block_eca(ctx, x, pre, spec):
    """nets/mobilenetV3.py:94-150 (Block_eca.forward); SeModule never called."""
    k, cin, exp, cout, act, _se, stride = spec
    out = _act(ctx.bn(ctx.conv(x, pre + "conv1"), pre + "bn1"), act)
    out = _act(ctx.bn(ctx.conv(out, pre + "conv2", stride, k // 2, exp), pre + "bn2"), act)
    out = eca(ctx, out, pre + "eca", "hsigmoid")
    out = ctx.bn(ctx.conv(out, pre + "conv3"), pre + "bn3")
    skip = x
    if stride == 1 and cin != cout:
        skip = ctx.bn(ctx.conv(x, pre + "skip.0"), pre + "skip.1")
    elif stride == 2 and cin != cout:
        s = ctx.bn(ctx.conv(x, pre + "skip.0", 2, 1, cin), pre + "skip.1")
        skip = ctx.bn(ctx.conv(s, pre + "skip.2"), pre + "skip.3")
    elif stride == 2:
        skip = ctx.bn(ctx.conv(x, pre + "skip.0", 2, 1, cin), pre + "skip.1")
    return _act(out + skip, act)


def mnv3_body(ctx, x):
    """MobileNetV3_Large_eca stem + layer1..3 -> (C3, C4, C5)."""
    x = kink(ctx.bn(ctx.conv(x, "body.conv1", 2, 1), "body.bn1"), "hswish")
    feats = []
    for li, layer in enumerate(MNV3_LAYERS):
        for bi, spec in enumerate(layer):
            x = block_eca(ctx, x, f"body.layer{li + 1}.{bi}.", spec)
        feats.append(x)
    return feats


def r50_body(ctx, x):
    """torchvision resnet50 stem + layer1..4, returning layer2/3/4."""
    x = kink(ctx.bn(ctx.conv(x, "body.conv1", 2, 3), "body.bn1"), "relu")
    x = maxpool(x)
    feats = []
    for li, (w, n, s) in enumerate(R50_LAYERS):
        for bi in range(n):
            pre = f"body.layer{li + 1}.{bi}."
            st = s if bi == 0 else 1
            out = kink(ctx.bn(ctx.conv(x, pre + "conv1"), pre + "bn1"), "relu")
            out = kink(ctx.bn(ctx.conv(out, pre + "conv2", st, 1), pre + "bn2"), "relu")
            out = ctx.bn(ctx.conv(out, pre + "conv3"), pre + "bn3")
            idn = x
            if bi == 0:
                idn = ctx.bn(ctx.conv(x, pre + "downsample.0", st), pre + "downsample.1")
            x = kink(out + idn, "relu")
        if li >= 1:
            feats.append(x)
    return feats


def psp(x, sizes):
    """PSPModule.forward (nets/retinaface_r.py:100-104)."""
    n, c = x.shape[:2]
    return torch.cat([F.adaptive_avg_pool2d(x, s).view(n, c, -1) for s in sizes], -1)


def nlm(ctx, x, pre, sizes=(1, 4, 8, 12)):
    """NLM.forward (nets/retinaface_r.py:124-152), scale=1."""
    B, _, h, w = x.shape
    q = ctx.conv(x, pre + "f_query")
    ch = q.shape[1]
    q = q.view(B, ch, -1).permute(0, 2, 1)
    k = psp(ctx.conv(x, pre + "f_key"), sizes)
    v = psp(ctx.conv(x, pre + "f_value"), sizes).permute(0, 2, 1)
    sim = F.softmax(torch.matmul(q, k) * (1 ** -.5), dim=-1)
    ctxv = torch.matmul(sim, v).permute(0, 2, 1).contiguous().view(B, ch, h, w)
    return ctx.conv(ctxv, pre + "W") + x


def conv_bn_act(ctx, x, pre, leaky, padding=0, act=True):
    y = ctx.bn(ctx.conv(x, pre + ".0", 1, padding), pre + ".1")
    return kink(y, "leaky", leaky) if act else y


def _up(x, ref, mode):
    if mode == "bicubic":  # train_mobilenetV3_ecagai.py:270,279
        return F.interpolate(x, size=[ref.shape[2], ref.shape[3]], mode="bicubic",
                             align_corners=True)
    return F.interpolate(x, size=[ref.shape[2], ref.shape[3]], mode="nearest")


def fpn(ctx, feats, leaky, nlm_name, pre="fpn.", sizes=(1, 4, 8, 12), up="nearest"):
    """FPN.forward (nets/retinaface_r.py:169-207); nlm_name=None is the plain
    FPN of nets/layers.py:83-119 (up-sample + add, no NLM); up="bicubic" is the
    BECA variant's FPN (train_mobilenetV3_ecagai.py:254-285)."""
    o1 = conv_bn_act(ctx, feats[0], pre + "output1", leaky)
    o2 = conv_bn_act(ctx, feats[1], pre + "output2", leaky)
    o3 = conv_bn_act(ctx, feats[2], pre + "output3", leaky)
    up3 = _up(o3, o2, up)
    if nlm_name is not None:
        up3 = nlm(ctx, up3, nlm_name, sizes)
    o2 = conv_bn_act(ctx, o2 + up3, pre + "merge2", leaky, 1)
    up2 = _up(o2, o1, up)
    if nlm_name is not None:
        up2 = nlm(ctx, up2, nlm_name, sizes)
    o1 = conv_bn_act(ctx, o1 + up2, pre + "merge1", leaky, 1)
    return [o1, o2, o3]


def ssh(ctx, x, pre, leaky):
    """SSH.forward (nets/layers.py:37-68)."""
    a = conv_bn_act(ctx, x, pre + "conv3X3", leaky, 1, act=False)
    b1 = conv_bn_act(ctx, x, pre + "conv5X5_1", leaky, 1)
    b = conv_bn_act(ctx, b1, pre + "conv5X5_2", leaky, 1, act=False)
    c1 = conv_bn_act(ctx, b1, pre + "conv7X7_2", leaky, 1)
    c = conv_bn_act(ctx, c1, pre + "conv7x7_3", leaky, 1, act=False)
    return kink(torch.cat([a, b, c], 1), "relu")


def heads(ctx, feats, mode):
    """Class/Bbox/Landmark heads + concat (nets/retinaface_r.py:17-57, 335-343)."""
    def run(kind, k):
        outs = []
        for i, f in enumerate(feats):
            o = ctx.conv(f, f"{kind}.{i}.conv1x1").permute(0, 2, 3, 1).contiguous()
            outs.append(o.view(o.shape[0], -1, k))
        return torch.cat(outs, 1)
    loc = run("BboxHead", 4)
    conf = run("ClassHead", 2)
    landm = run("LandmarkHead", 10)
    if mode != "train":
        conf = F.softmax(conf, dim=-1)
    return loc, conf, landm


def retinaface_mnv3(P, x, mode="eval", train_bn=False):
    """JABD-MobileNetV3 RetinaFace.forward (nets/retinaface_r.py:304-343)."""
    ctx = Ctx(P, train_bn)
    c3, c4, c5 = mnv3_body(ctx, x)
    feats = [eca(ctx, c3, "eca_40", "sigmoid"), eca(ctx, c4, "eca_80", "sigmoid"),
             eca(ctx, c5, "eca_160", "sigmoid")]
    f = fpn(ctx, feats, 0.1, "fpn.nlm.")
    f = [ssh(ctx, eca(ctx, f[i], "eca_fpn", "sigmoid"), f"ssh{i + 1}.", 0.1) for i in range(3)]
    return heads(ctx, f, mode)


def retinaface_r50(P, x, mode="eval", train_bn=False):
    """RetinaFace-R50 + ECA + NLM (nets/retinaface_eca_nonlocal.py:314-359)."""
    ctx = Ctx(P, train_bn)
    c3, c4, c5 = r50_body(ctx, x)
    feats = [eca(ctx, c3, "eca_64", "sigmoid"), eca(ctx, c4, "eca_128", "sigmoid"),
             eca(ctx, c5, "eca_256", "sigmoid")]
    f = fpn(ctx, feats, 0.0, "fpn.Nlm.")
    f = [ssh(ctx, eca(ctx, f[i], "eca_fpn", "sigmoid"), f"ssh{i + 1}.", 0.0) for i in range(3)]
    return heads(ctx, f, mode)


def retinaface_mnv3_beca(P, x, mode="eval", train_bn=False):
    """JABD-MobileNetV3-BECA (train_mobilenetV3_ecagai.py:319-435): the same
    body, BECA gates (std pool -> Conv1d -> Hardsigmoid, :286-316) for
    eca_40/80/160 and eca_fpn, FPN with bicubic align_corners up-sampling and
    NLM(40) of ch=40 with PSP (1, 3, 6, 8) (:161-234)."""
    ctx = Ctx(P, train_bn)
    c3, c4, c5 = mnv3_body(ctx, x)
    feats = [stdv_eca(ctx, c3, "eca_40."), stdv_eca(ctx, c4, "eca_80."),
             stdv_eca(ctx, c5, "eca_160.")]
    f = fpn(ctx, feats, 0.1, "fpn.nlm.", sizes=(1, 3, 6, 8), up="bicubic")
    f = [ssh(ctx, stdv_eca(ctx, f[i], "eca_fpn."), f"ssh{i + 1}.", 0.1) for i in range(3)]
    return heads(ctx, f, mode)


# nets/mobilenetV3.py:216-228 (MobileNetV3_Small.bneck; every block has an SE
# flag), split where the detector body taps it (stride 8 / 16 / 32)
MNV3_SMALL_LAYERS = [
    [(3, 16, 16, 16, "relu", True, 2), (3, 16, 72, 24, "relu", False, 2),
     (3, 24, 88, 24, "relu", False, 1)],
    [(5, 24, 96, 40, "hswish", True, 2), (5, 40, 240, 40, "hswish", True, 1),
     (5, 40, 240, 40, "hswish", True, 1), (5, 40, 120, 48, "hswish", True, 1),
     (5, 48, 144, 48, "hswish", True, 1)],
    [(5, 48, 288, 96, "hswish", True, 2), (5, 96, 576, 96, "hswish", True, 1),
     (5, 96, 576, 96, "hswish", True, 1)],
]


def retinaface_mnv3_small(P, x, mode="eval", train_bn=False):
    """MobileNetV3_Small body (Block with SE / no gate, nets/mobilenetV3.py:35-91,
    210-229) tapped after bneck[2], [7], [10], under the JABD head of
    nets/retinaface_r.py:304-343 (eca_24/48/96)."""
    ctx = Ctx(P, train_bn)
    x = kink(ctx.bn(ctx.conv(x, "body.conv1", 2, 1), "body.bn1"), "hswish")
    feats = []
    i = 0
    for layer in MNV3_SMALL_LAYERS:
        for spec in layer:
            x = block(ctx, x, f"body.bneck.{i}.", spec, "se" if spec[5] else "none")
            i += 1
        feats.append(x)
    feats = [eca(ctx, f, n, "sigmoid") for f, n in zip(feats, ("eca_24", "eca_48", "eca_96"))]
    f = fpn(ctx, feats, 0.1, "fpn.nlm.")
    f = [ssh(ctx, eca(ctx, f[i], "eca_fpn", "sigmoid"), f"ssh{i + 1}.", 0.1) for i in range(3)]
    return heads(ctx, f, mode)


# ----------------------------------------------------------------------------- module-level
# restatements for the module surface (nets/* forwards run one by one)
def se(ctx, x, pre):
    """SeModule.forward (nets/mobilenetV3.py:18-32): x * hsigmoid(conv(relu(bn(conv(GAP(x))))))."""
    y = F.adaptive_avg_pool2d(x, 1)
    y = kink(ctx.bn(ctx.conv(y, pre + "se.1"), pre + "se.2"), "relu")
    y = kink(ctx.conv(y, pre + "se.4"), "hsigmoid")
    return x * y


def stdv_eca(ctx, x, pre):
    """eca_block_G.forward (nets/mobilenetV3.py:350-377): population std over H*W
    (mean_channels / stdv_channels), Conv1d over channels, Hardsigmoid, x*y."""
    w = ctx.P[pre + "conv.weight"]
    k = w.shape[-1]
    mean = x.sum(3, keepdim=True).sum(2, keepdim=True) / (x.shape[2] * x.shape[3])
    var = (x - mean).pow(2).sum(3, keepdim=True).sum(2, keepdim=True) / (x.shape[2] * x.shape[3])
    y = var.pow(0.5)
    y = F.conv1d(y.squeeze(-1).transpose(-1, -2), w, padding=(k - 1) // 2)
    y = kink(y.transpose(-1, -2).unsqueeze(-1), "hsigmoid")
    return x * y


def block(ctx, x, pre, spec, gate="eca"):
    """Block (gate "se"/"none", nets/mobilenetV3.py:35-91), Block_eca ("eca",
    :94-150), Block_eca_G ("beca", :152-208)."""
    if gate == "eca":
        return block_eca(ctx, x, pre, spec)
    k, cin, exp, cout, act, _se, stride = spec
    out = _act(ctx.bn(ctx.conv(x, pre + "conv1"), pre + "bn1"), act)
    out = _act(ctx.bn(ctx.conv(out, pre + "conv2", stride, k // 2, exp), pre + "bn2"), act)
    if gate == "se":
        out = se(ctx, out, pre + "se.")
    elif gate == "beca":
        out = stdv_eca(ctx, out, pre + "eca.")
    out = ctx.bn(ctx.conv(out, pre + "conv3"), pre + "bn3")
    skip = x
    if stride == 1 and cin != cout:
        skip = ctx.bn(ctx.conv(x, pre + "skip.0"), pre + "skip.1")
    elif stride == 2 and cin != cout:
        s = ctx.bn(ctx.conv(x, pre + "skip.0", 2, 1, cin), pre + "skip.1")
        skip = ctx.bn(ctx.conv(s, pre + "skip.2"), pre + "skip.3")
    elif stride == 2:
        skip = ctx.bn(ctx.conv(x, pre + "skip.0", 2, 1, cin), pre + "skip.1")
    return _act(out + skip, act)


def bn1d(ctx, x, name):
    P = ctx.P
    return F.batch_norm(x, P[name + ".running_mean"], P[name + ".running_var"],
                        P[name + ".weight"], P[name + ".bias"], ctx.train, ctx.momentum, ctx.eps)


def mobilenetv3(P, x, stages, train_bn=False):
    """MobileNetV3_{Small,Large,Large_eca,...}.forward (nets/mobilenetV3.py:257-265,
    510-522): stem, stages = [(prefix, [(spec, gate), ...]), ...], conv2+bn2+hs,
    GAP, linear3+bn3+hs (dropout: identity in eval), linear4."""
    ctx = Ctx(P, train_bn)
    x = kink(ctx.bn(ctx.conv(x, "conv1", 2, 1), "bn1"), "hswish")
    for pre, blocks in stages:
        for bi, (spec, gate) in enumerate(blocks):
            x = block(ctx, x, f"{pre}.{bi}.", spec, gate)
    x = kink(ctx.bn(ctx.conv(x, "conv2"), "bn2"), "hswish")
    x = F.adaptive_avg_pool2d(x, 1).flatten(1)
    x = kink(bn1d(ctx, F.linear(x, P["linear3.weight"]), "bn3"), "hswish")
    return F.linear(x, P["linear4.weight"], P["linear4.bias"])


def mobilenetv1_stage(ctx, x, pre, specs):
    """conv_bn / conv_dw Sequentials (nets/mobilenet025.py:3-19): specs =
    [(kind, cin, cout, stride), ...]."""
    for i, (kind, cin, cout, stride) in enumerate(specs):
        p = f"{pre}.{i}."
        if kind == "bn":
            x = kink(ctx.bn(ctx.conv(x, p + "0", stride, 1), p + "1"), "leaky", 0.1)
        else:
            x = kink(ctx.bn(ctx.conv(x, p + "0", stride, 1, cin), p + "1"), "leaky", 0.1)
            x = kink(ctx.bn(ctx.conv(x, p + "3"), p + "4"), "leaky", 0.1)
    return x


MNV1_STAGES = [
    [("bn", 3, 8, 2), ("dw", 8, 16, 1), ("dw", 16, 32, 2), ("dw", 32, 32, 1),
     ("dw", 32, 64, 2), ("dw", 64, 64, 1)],
    [("dw", 64, 128, 2)] + [("dw", 128, 128, 1)] * 5,
    [("dw", 128, 256, 2), ("dw", 256, 256, 1)],
]


def resnet_classifier(P, x, layers=R50_LAYERS, train_bn=False):
    """ResNet._forward_impl (nets/resnet_pytorch_r.py:232-250) for Bottleneck nets."""
    ctx = Ctx(P, train_bn)
    P2 = {("body." + k): v for k, v in P.items()}
    c = Ctx(P2, train_bn)
    feats = r50_body(c, x)
    x = F.adaptive_avg_pool2d(feats[-1], 1).flatten(1)
    return F.linear(x, ctx.P["fc.weight"], ctx.P["fc.bias"])
