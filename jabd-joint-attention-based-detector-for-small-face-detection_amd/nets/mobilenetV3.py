"""MobileNetV3 family — drop-in for the reference nets/mobilenetV3.py:1-731
(same class names, constructor signatures and state_dict keys).

Every module runs libjabd kernels (jabd_amd/modules.py):
  * a block (Block_eca :94-150, Block :35-91 with SE, Block_eca_G :152-208
    with the std-pooled BECA gate) is one fused plan — eval: expand 1x1 +
    depthwise in one kernel, the channel gate as a per-(image, channel)
    scale the project GEMM applies on load, the skip K-concatenated or added
    in its epilogue; training: the autograd graph of jabd_amd/train.py;
  * the backbones' forward (stem, stages, classifier tail) chains them;
  * inside RetinaFace.forward the same block packs run as part of the fused
    detector plan.
As in the reference, Block_eca builds a SeModule it never applies (:110 vs
:140-150).
"""
import math

import torch
import torch.nn as nn
from torch.nn import init

from jabd_amd import modules as M
from jabd_amd import train as T
from jabd_amd.engine import _MNv3Block
from jabd_amd.hipmodule import HipModule


class hswish(HipModule):
    """x * relu6(x + 3) / 6 (reference :6-9)."""

    def forward(self, x):
        with M._Mode(self):
            return M.activation(x, "hswish")


class hsigmoid(HipModule):
    """relu6(x + 3) / 6 (reference :12-15)."""

    def forward(self, x):
        with M._Mode(self):
            return M.activation(x, "hsigmoid")


def _act_module(act):
    """The reference passes torch activation classes (nn.ReLU / nn.Hardswish);
    build the HIP subclass with the same name and keys."""
    return {nn.ReLU: M.ReLU, nn.Hardswish: M.Hardswish}.get(act, act)


def _act_name(act):
    if act in (nn.ReLU, M.ReLU):
        return "relu"
    if act in (nn.Hardswish, M.Hardswish, hswish):
        return "hswish"
    raise NotImplementedError(f"block activation {act}")


class SeModule(HipModule):
    """x * hsigmoid(conv(relu(bn(conv(GAP(x)))))) (reference :18-32)."""

    def __init__(self, in_size, reduction=4):
        super().__init__()
        mid = max(in_size // reduction, 8)
        self.se = nn.Sequential(
            M.AdaptiveAvgPool2d(1),
            M.Conv2d(in_size, mid, kernel_size=1, bias=False),
            M.BatchNorm2d(mid),
            M.ReLU(inplace=True),
            M.Conv2d(mid, in_size, kernel_size=1, bias=False),
            M.Hardsigmoid(),
        )

    def forward(self, x):
        xh = M.nhwc(x, "SeModule input").contiguous()
        with M._Mode(self):
            if self.training:
                s = M.se_scale_train(self, xh)
            else:
                s = M.se_scale_eval(self, xh, self)
            return M.nchw(M.ScaleFn.apply(xh, s))


def eca_kernel_size(channel, b=1, gamma=2):
    k = int(abs((math.log(channel, 2) + b) / gamma))
    return k if k % 2 else k + 1


class eca_block(HipModule):
    """In-block ECA (Hardsigmoid gate) — reference :332-348."""
    gate = "hsigmoid"

    def __init__(self, channel, b=1, gamma=2):
        super().__init__()
        k = eca_kernel_size(channel, b, gamma)
        self.avg_pool = M.AdaptiveAvgPool2d(1)
        self.conv = nn.Conv1d(1, 1, kernel_size=k, padding=(k - 1) // 2, bias=False)
        self.sigmoid = M.Sigmoid()
        self.Hsigmoid = M.Hardsigmoid()

    def forward(self, x):
        with M._Mode(self):
            return M.nchw(M.EcaScaleFn.apply(M.nhwc(x, "eca_block input").contiguous(),
                                             self.conv.weight, self.gate))


def mean_channels(F):
    """Per-channel spatial mean [B, C, 1, 1] (reference :350-353)."""
    B, C = F.shape[0], F.shape[1]
    return M.global_avg_pool(M.nhwc(F).contiguous()).view(B, 1, 1, C).permute(0, 3, 1, 2)


def stdv_channels(F):
    """Per-channel spatial population std [B, C, 1, 1] (reference :356-359)."""
    B, C = F.shape[0], F.shape[1]
    with torch.no_grad():
        xh = M.nhwc(F).contiguous()
        stats = torch.empty((4, B * C), dtype=torch.float32, device=F.device)
        w = torch.zeros(1, dtype=torch.float32, device=F.device)
        P = xh.shape[1] * xh.shape[2]
        from jabd_amd.ops import beca_part
        part = beca_part(B, P, C, F.device)
        M.call("jabd_beca_fwd_f32", xh.data_ptr(), B, P, C, w.data_ptr(), 1, None,
               stats.data_ptr(), part.data_ptr(), part.numel(), M._st())
    return stats[1].view(B, C, 1, 1)


class eca_block_G(HipModule):
    """Contrast ECA (BECA): x * hardsigmoid(conv1d(std_hw(x))) (reference :361-377)."""

    def __init__(self, channel, b=1, gamma=2):
        super().__init__()
        k = eca_kernel_size(channel, b, gamma)
        self.avg_pool = M.AdaptiveAvgPool2d(1)
        self.conv = nn.Conv1d(1, 1, kernel_size=k, padding=(k - 1) // 2, bias=False)
        self.sigmoid = M.Sigmoid()
        self.Hsigmoid = M.Hardsigmoid()
        self.contrast = stdv_channels

    def forward(self, x):
        from jabd_amd.ops import BecaFn
        with M._Mode(self):
            xh = M.nhwc(x, "eca_block_G input").contiguous()
            return M.nchw(BecaFn.apply(xh, self.conv.weight.reshape(-1)))


def _skip(stride, in_size, out_size):
    if stride == 1 and in_size != out_size:
        return nn.Sequential(M.Conv2d(in_size, out_size, kernel_size=1, bias=False),
                             M.BatchNorm2d(out_size))
    if stride == 2 and in_size != out_size:
        return nn.Sequential(
            M.Conv2d(in_size, in_size, kernel_size=3, groups=in_size, stride=2, padding=1,
                     bias=False),
            M.BatchNorm2d(in_size),
            M.Conv2d(in_size, out_size, kernel_size=1, bias=True),
            M.BatchNorm2d(out_size))
    if stride == 2 and in_size == out_size:
        return nn.Sequential(
            M.Conv2d(in_size, out_size, kernel_size=3, groups=in_size, stride=2, padding=1,
                     bias=False),
            M.BatchNorm2d(out_size))
    return None


class _BlockBase(HipModule):
    """expand 1x1 -> depthwise kxk -> gate -> project 1x1 (+skip) -> act."""
    gate_kind = "eca"

    def _build(self, kernel_size, in_size, expand_size, out_size, act, se, stride):
        self.stride = stride
        self.kernel_size = kernel_size
        self.in_size, self.expand_size, self.out_size = in_size, expand_size, out_size
        self.act_name = _act_name(act)
        act = _act_module(act)
        self.conv1 = M.Conv2d(in_size, expand_size, kernel_size=1, bias=False)
        self.bn1 = M.BatchNorm2d(expand_size)
        self.act1 = act(inplace=True)
        self.conv2 = M.Conv2d(expand_size, expand_size, kernel_size=kernel_size, stride=stride,
                              padding=kernel_size // 2, groups=expand_size, bias=False)
        self.bn2 = M.BatchNorm2d(expand_size)
        self.act2 = act(inplace=True)
        self.se = SeModule(expand_size) if se else nn.Identity()

    def _tail(self, out_size, act, stride, in_size):
        act = _act_module(act)
        self.conv3 = M.Conv2d(self.expand_size, out_size, kernel_size=1, bias=False)
        self.bn3 = M.BatchNorm2d(out_size)
        self.act3 = act(inplace=True)
        self.skip = _skip(stride, in_size, out_size)

    def forward(self, x):
        xh = M.nhwc(x, f"{type(self).__name__} input").contiguous()
        if self.training:
            return M.nchw(T._mnv3_block(self, xh))
        blk = self._jabd_cached(x.device, lambda: _MNv3Block(self))
        with torch.no_grad():
            return M.nchw(blk.forward(xh))


class Block(_BlockBase):
    """MobileNetV3 block with the SE gate applied (reference :35-91)."""

    def __init__(self, kernel_size, in_size, expand_size, out_size, act, se, stride):
        super().__init__()
        self._build(kernel_size, in_size, expand_size, out_size, act, se, stride)
        self.gate_kind = "se" if se else "none"
        self._tail(out_size, act, stride, in_size)


class Block_eca(_BlockBase):
    """MobileNetV3 block with the in-block ECA gate (reference :94-150)."""

    def __init__(self, kernel_size, in_size, expand_size, out_size, act, se, stride):
        super().__init__()
        self._build(kernel_size, in_size, expand_size, out_size, act, se, stride)
        self.eca = eca_block(expand_size)
        self._tail(out_size, act, stride, in_size)


class Block_eca_G(_BlockBase):
    """MobileNetV3 block with the contrast (std-pooled) ECA gate (reference :152-208)."""
    gate_kind = "beca"

    def __init__(self, kernel_size, in_size, expand_size, out_size, act, se, stride):
        super().__init__()
        self._build(kernel_size, in_size, expand_size, out_size, act, se, stride)
        self.eca = eca_block_G(expand_size)
        self._tail(out_size, act, stride, in_size)


def _init_params(module):
    for m in module.modules():
        if isinstance(m, nn.Conv2d):
            init.kaiming_normal_(m.weight, mode="fan_out")
            if m.bias is not None:
                init.constant_(m.bias, 0)
        elif isinstance(m, nn.BatchNorm2d):
            init.constant_(m.weight, 1)
            init.constant_(m.bias, 0)
        elif isinstance(m, nn.Linear):
            init.normal_(m.weight, std=0.001)
            if m.bias is not None:
                init.constant_(m.bias, 0)


class _MobileNetV3(HipModule):
    """Stem 3x3/s2 + BN + act, the stages, then conv 1x1 + BN + act, GAP,
    Linear + BN1d + act, Dropout, Linear (reference :210-266 and kin)."""
    stages = ()

    def _stem(self, act):
        self.conv1 = M.Conv2d(3, 16, kernel_size=3, stride=2, padding=1, bias=False)
        self.bn1 = M.BatchNorm2d(16)
        self.hs1 = _act_module(act)(inplace=True)

    def _classifier(self, cin, cmid, num_classes, act):
        act = _act_module(act)
        self.conv2 = M.Conv2d(cin, cmid, kernel_size=1, stride=1, padding=0, bias=False)
        self.bn2 = M.BatchNorm2d(cmid)
        self.hs2 = act(inplace=True)
        self.gap = M.AdaptiveAvgPool2d(1)
        self.linear3 = M.Linear(cmid, 1280, bias=False)
        self.bn3 = M.BatchNorm1d(1280)
        self.hs3 = act(inplace=True)
        self.drop = nn.Dropout(0.2)
        self.linear4 = M.Linear(1280, num_classes)

    def init_params(self):
        _init_params(self)

    def features(self, x):
        with M._Mode(self):
            out = M.nchw(M.conv_bn_act(self, self.conv1, self.bn1, x, *M.act_of(self.hs1)))
        for name in self.stages:
            out = getattr(self, name)(out)
        return out

    def forward(self, x):
        out = self.features(x)
        with M._Mode(self):
            out = M.conv_bn_act(self, self.conv2, self.bn2, out, *M.act_of(self.hs2))
            out = M.global_avg_pool(out)
        out = self.drop(self.hs3(self.bn3(self.linear3(out))))
        return self.linear4(out)


def _seq(block, specs, act):
    return nn.Sequential(*[block(k, i, e, o, (a if a is nn.ReLU else act), se, s)
                           for (k, i, e, o, a, se, s) in specs])


_R, _H = nn.ReLU, nn.Hardswish
# (kernel, in, expand, out, act, se, stride) per layer — reference :459-481
LARGE_ECA_LAYERS = (
    ((3, 16, 16, 16, _R, False, 1), (3, 16, 64, 24, _R, False, 2),
     (3, 24, 72, 24, _R, False, 1), (5, 24, 72, 40, _R, True, 2),
     (5, 40, 120, 40, _R, True, 1), (5, 40, 120, 40, _R, True, 1)),
    ((3, 40, 240, 80, _H, False, 2), (3, 80, 200, 80, _H, False, 1),
     (3, 80, 184, 80, _H, False, 1), (3, 80, 184, 80, _H, False, 1)),
    ((3, 80, 480, 112, _H, True, 1), (3, 112, 672, 112, _H, True, 1),
     (5, 112, 672, 160, _H, True, 2), (5, 160, 672, 160, _H, True, 1),
     (5, 160, 960, 160, _H, True, 1)),
)
# reference :216-228
SMALL_LAYERS = (
    (3, 16, 16, 16, _R, True, 2), (3, 16, 72, 24, _R, False, 2), (3, 24, 88, 24, _R, False, 1),
    (5, 24, 96, 40, _H, True, 2), (5, 40, 240, 40, _H, True, 1), (5, 40, 240, 40, _H, True, 1),
    (5, 40, 120, 48, _H, True, 1), (5, 48, 144, 48, _H, True, 1), (5, 48, 288, 96, _H, True, 2),
    (5, 96, 576, 96, _H, True, 1), (5, 96, 576, 96, _H, True, 1),
)


class MobileNetV3_Small(_MobileNetV3):
    """Reference :210-265: 11 SE blocks in one `bneck` Sequential."""
    stages = ("bneck",)

    def __init__(self, num_classes=1000, act=nn.Hardswish):
        super().__init__()
        self._stem(act)
        self.bneck = _seq(Block, SMALL_LAYERS, act)
        self._classifier(96, 576, num_classes, act)
        self.init_params()


class MobileNetV3_Large(_MobileNetV3):
    """Reference :268-330: the 15 SE blocks in one `bneck` Sequential."""
    stages = ("bneck",)

    def __init__(self, num_classes=1000, act=nn.Hardswish):
        super().__init__()
        self._stem(act)
        self.bneck = _seq(Block, sum(LARGE_ECA_LAYERS, ()), act)
        self._classifier(160, 960, num_classes, act)
        self.init_params()


class MobileNetV3_Large_eca(_MobileNetV3):
    """Reference :452-522: Block_eca stages layer1..3 (C3/C4/C5 = 40/80/160)."""
    stages = ("layer1", "layer2", "layer3")

    def __init__(self, num_classes=1000, act=nn.Hardswish):
        super().__init__()
        self._stem(act)
        for li, specs in enumerate(LARGE_ECA_LAYERS):
            setattr(self, f"layer{li + 1}", _seq(Block_eca, specs, act))
        self._classifier(160, 960, num_classes, act)
        _init_params(self)


class MobileNetV3_Large_change(_MobileNetV3):
    """Reference :524-595: the Large layout in layer1..3 of SE Blocks."""
    stages = ("layer1", "layer2", "layer3")

    def __init__(self, num_classes=1000, act=nn.Hardswish):
        super().__init__()
        self._stem(act)
        for li, specs in enumerate(LARGE_ECA_LAYERS):
            setattr(self, f"layer{li + 1}", _seq(Block, specs, act))
        self._classifier(160, 960, num_classes, act)
        self.init_params()


# reference :380-436: Block_eca with Block_eca_G at layer1[3] and layer2[2]
_ECAG_AT = {(0, 3), (1, 2)}


class MobileNetV3_Large_ecaG(_MobileNetV3):
    stages = ("layer1", "layer2", "layer3")

    def __init__(self, num_classes=1000, act=nn.Hardswish):
        super().__init__()
        self._stem(act)
        for li, specs in enumerate(LARGE_ECA_LAYERS):
            blocks = [(Block_eca_G if (li, bi) in _ECAG_AT else Block_eca)(
                k, i, e, o, (a if a is nn.ReLU else act), se, s)
                for bi, (k, i, e, o, a, se, s) in enumerate(specs)]
            setattr(self, f"layer{li + 1}", nn.Sequential(*blocks))
        self._classifier(160, 960, num_classes, act)
        self.init_params()


class MobileNetV3_Large_4(_MobileNetV3):
    """Reference :597-668: four stages (strides 8/16/16/32) of SE Blocks."""
    stages = ("layer1", "layer2", "layer3", "layer4")

    def __init__(self, num_classes=1000, act=nn.Hardswish):
        super().__init__()
        self._stem(act)
        L = sum(LARGE_ECA_LAYERS, ())
        for li, (lo, hi) in enumerate(((0, 4), (4, 7), (7, 10), (10, 15))):
            setattr(self, f"layer{li + 1}", _seq(Block, L[lo:hi], act))
        self._classifier(160, 960, num_classes, act)
        self.init_params()


def conv_bn(inp, oup, stride=1, leaky=0.1):
    """Reference :715-720."""
    return M.FusedSequential(M.Conv2d(inp, oup, 3, stride, 1, bias=False), M.BatchNorm2d(oup),
                             M.LeakyReLU(negative_slope=leaky, inplace=True))


def conv_dw(inp, oup, stride=1, leaky=0.1):
    """Depthwise 3x3 + BN + leaky, pointwise 1x1 + BN + leaky (reference :723-731)."""
    return M.FusedSequential(
        M.Conv2d(inp, inp, 3, stride, 1, groups=inp, bias=False), M.BatchNorm2d(inp),
        M.LeakyReLU(negative_slope=leaky, inplace=True),
        M.Conv2d(inp, oup, 1, 1, 0, bias=False), M.BatchNorm2d(oup),
        M.LeakyReLU(negative_slope=leaky, inplace=True))


class MobileNetV1(HipModule):
    """MobileNetV1-0.25 (reference :670-712 and nets/mobilenet025.py:21-64).
    The reference's forward names nonexistent `stage1..3`; this one runs the
    defined layer1..3 -> GAP -> fc."""

    def __init__(self):
        super().__init__()
        self.layer1 = nn.Sequential(conv_bn(3, 8, 2, leaky=0.1), conv_dw(8, 16, 1),
                                    conv_dw(16, 32, 2), conv_dw(32, 32, 1),
                                    conv_dw(32, 64, 2), conv_dw(64, 64, 1))
        self.layer2 = nn.Sequential(conv_dw(64, 128, 2), *[conv_dw(128, 128, 1) for _ in range(5)])
        self.layer3 = nn.Sequential(conv_dw(128, 256, 2), conv_dw(256, 256, 1))
        self.avg = M.AdaptiveAvgPool2d((1, 1))
        self.fc = M.Linear(256, 1000)

    def forward(self, x):
        x = self.layer3(self.layer2(self.layer1(x)))
        with M._Mode(self):
            x = M.global_avg_pool(M.nhwc(x).contiguous())
        return self.fc(x)
