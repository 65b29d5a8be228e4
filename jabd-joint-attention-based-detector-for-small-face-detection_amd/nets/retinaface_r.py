"""JABD-MobileNetV3 RetinaFace — drop-in for the reference
nets/retinaface_r.py:17-343 (same class names, constructor signatures and
state_dict keys).

`RetinaFace.forward(x[B,3,H,W] fp32 GPU)` runs the whole detector as one fused
HIP plan (jabd_amd/engine.py in eval mode, jabd_amd/train.py's autograd graph
in training mode) and returns (loc [B,A,4], conf [B,A,2] (softmaxed iff
mode != 'train'), landm [B,A,10]).  Every other class here also has a forward
of its own over libjabd kernels (jabd_amd/modules.py), so a script that
composes them itself — as train_mobilenetV3_ecagai.py:319-435 does — runs on
the same kernels.
"""
import math
from collections import OrderedDict

import torch
import torch.nn as nn

from jabd_amd import modules as M
from jabd_amd import train as T
from jabd_amd.engine import NlmPack, retinaface_forward
from jabd_amd.hipmodule import HipModule
from nets._getter import IntermediateLayerGetter
from nets.layers import SSH, conv_bn, conv_bn1X1, conv_bn_no_relu, fpn_forward  # noqa: F401
from nets.mobilenetV3 import MobileNetV3_Large_eca, MobileNetV3_Small


class _Head1x1(HipModule):
    """1x1 conv (with bias) -> permute(0,2,3,1) -> view(B, -1, k): the NHWC
    conv output already is the permuted tensor (no copy)."""
    k = 1

    def forward(self, x):
        xh = M.nhwc(x, f"{type(self).__name__} input")
        with M._Mode(self):
            if self.training:
                y = T.ConvFn.apply(xh, self.conv1x1.weight, self.conv1x1.bias, 1, 0, False)
            else:
                pk = self._jabd_cached(x.device, lambda: M.F.pack_conv(self.conv1x1))
                y = M.F.conv(xh, pk)
        return y.view(y.shape[0], -1, self.k)


class ClassHead(_Head1x1):
    k = 2

    def __init__(self, inchannels=512, num_anchors=2):
        super().__init__()
        self.num_anchors = num_anchors
        self.conv1x1 = M.Conv2d(inchannels, num_anchors * 2, kernel_size=(1, 1), stride=1,
                                padding=0)


class BboxHead(_Head1x1):
    k = 4

    def __init__(self, inchannels=512, num_anchors=2):
        super().__init__()
        self.conv1x1 = M.Conv2d(inchannels, num_anchors * 4, kernel_size=(1, 1), stride=1,
                                padding=0)


class LandmarkHead(_Head1x1):
    k = 10

    def __init__(self, inchannels=512, num_anchors=2):
        super().__init__()
        self.conv1x1 = M.Conv2d(inchannels, num_anchors * 10, kernel_size=(1, 1), stride=1,
                                padding=0)


class PSPModule(HipModule):
    """Adaptive-average pools at `sizes`, concatenated: [n, c, S] (reference :85-104)."""

    def __init__(self, sizes=(1, 3, 6, 8), dimension=2):
        super().__init__()
        if dimension != 2:
            raise NotImplementedError("PSPModule: the 2-D pools are the ones JABD uses")
        self.sizes = tuple(sizes)
        self.stages = nn.ModuleList([M.AdaptiveAvgPool2d((s, s)) for s in sizes])

    def forward(self, feats):
        with M._Mode(self):
            out = M.AdaptivePoolFn.apply(M.nhwc(feats, "PSPModule input"), self.sizes)
        return out.permute(0, 2, 1)


class NLM(HipModule):
    """PSP-pooled non-local block, the CSAF attention (reference :107-152):
    x + W(softmax(q(x) . psp(k(x))) . psp(v(x)))."""

    def __init__(self, in_channels, scale=1, psp_size=(1, 4, 8, 12), ch=4):
        super().__init__()
        if scale != 1:
            raise NotImplementedError("NLM scale > 1 is not used by any JABD model")
        self.scale, self.in_channels, self.ch = scale, in_channels, ch
        self.pool = nn.MaxPool2d(kernel_size=(scale, scale))
        self.f_query = M.Conv2d(in_channels, ch, kernel_size=1)
        self.f_key = M.Conv2d(in_channels, ch, kernel_size=1)
        self.f_value = M.Conv2d(in_channels, ch, kernel_size=1)
        self.psp = PSPModule(psp_size)
        self.W = M.Conv2d(ch, in_channels, kernel_size=1)
        nn.init.constant_(self.W.weight, 0)
        nn.init.constant_(self.W.bias, 0)

    def forward(self, x):
        xh = M.nhwc(x, "NLM input").contiguous()
        if self.training:
            return M.nchw(T.nlm_train(self, xh))
        pk = self._jabd_cached(x.device, lambda: NlmPack(self))
        with torch.no_grad():
            return M.nchw(pk.forward(xh))


class FPN(HipModule):
    """Laterals, nearest up-sample -> shared NLM -> add, merges (reference :154-207)."""

    def __init__(self, in_channels_list, out_channels):
        super().__init__()
        self.leaky = 0.1 if out_channels <= 64 else 0.0
        self.output1 = conv_bn1X1(in_channels_list[0], out_channels, stride=1, leaky=self.leaky)
        self.output2 = conv_bn1X1(in_channels_list[1], out_channels, stride=1, leaky=self.leaky)
        self.output3 = conv_bn1X1(in_channels_list[2], out_channels, stride=1, leaky=self.leaky)
        self.merge1 = conv_bn(out_channels, out_channels, leaky=self.leaky)
        self.merge2 = conv_bn(out_channels, out_channels, leaky=self.leaky)
        self.nlm = NLM(40)

    def forward(self, inputs):
        return fpn_forward(self, inputs, self.nlm)


class eca_block(HipModule):
    """Head ECA with a Sigmoid gate (reference :208-224): x * sigmoid(conv1d(GAP(x)))."""
    gate = "sigmoid"

    def __init__(self, channel, b=1, gamma=2):
        super().__init__()
        k = int(abs((math.log(channel, 2) + b) / gamma))
        k = k if k % 2 else k + 1
        self.avg_pool = M.AdaptiveAvgPool2d(1)
        self.conv = nn.Conv1d(1, 1, kernel_size=k, padding=(k - 1) // 2, bias=False)
        self.sigmoid = M.Sigmoid()
        self.Hsigmoid = M.Hardsigmoid()

    def forward(self, x):
        with M._Mode(self):
            return M.nchw(M.EcaScaleFn.apply(M.nhwc(x, "eca_block input").contiguous(),
                                             self.conv.weight, self.gate))


class RetinaFace(HipModule):
    def __init__(self, cfg=None, pretrained=False, mode="train"):
        super().__init__()
        if cfg["name"] != "mobilenet0.25":
            raise ValueError("nets.retinaface_r.RetinaFace is the JABD-MobileNetV3 model "
                             "(cfg_mnet); use nets.retinaface_eca_nonlocal for ResNet-50")
        if pretrained:
            raise RuntimeError("the reference's pretrained backbone checkpoint is not shipped")
        backbone = MobileNetV3_Large_eca()
        self.body = IntermediateLayerGetter(backbone, cfg["return_layers"])
        c = cfg["in_channel"]
        self.fpn = FPN([c * 2, c * 4, c * 8], cfg["out_channel"])
        self.ssh1 = SSH(cfg["out_channel"], cfg["out_channel"])
        self.ssh2 = SSH(cfg["out_channel"], cfg["out_channel"])
        self.ssh3 = SSH(cfg["out_channel"], cfg["out_channel"])
        oc = cfg["out_channel"]
        self.ClassHead = nn.ModuleList([ClassHead(oc, 2) for _ in range(3)])
        self.BboxHead = nn.ModuleList([BboxHead(oc, 2) for _ in range(3)])
        self.LandmarkHead = nn.ModuleList([LandmarkHead(oc, 2) for _ in range(3)])
        self.eca_40 = eca_block(40)
        self.eca_80 = eca_block(80)
        self.eca_160 = eca_block(160)
        self.eca_fpn = eca_block(40)
        self.mode = mode
        self.cfg = cfg

    def forward(self, inputs):
        return retinaface_forward(self, "mnv3", inputs)


class MobileNetV3SmallBody(HipModule):
    """MobileNetV3_Small's stem + `bneck` (reference nets/mobilenetV3.py:210-229)
    as a detector body.  The reference has no detector wiring for it (its
    blocks sit in one Sequential, which IntermediateLayerGetter cannot tap);
    this taps bneck[2] (stride 8, 24 ch), bneck[7] (stride 16, 48 ch) and
    bneck[10] (stride 32, 96 ch) — the last block of each resolution — and
    returns them as IntermediateLayerGetter would.  Keys stay the
    classifier's (`conv1`, `bn1`, `bneck.N...`) so its checkpoint loads."""
    splits = (3, 8, 11)

    def __init__(self, backbone):
        super().__init__()
        self.conv1, self.bn1, self.hs1 = backbone.conv1, backbone.bn1, backbone.hs1
        self.bneck = backbone.bneck

    def stages(self):
        b = list(self.bneck)
        lo = 0
        out = []
        for hi in self.splits:
            out.append(b[lo:hi])
            lo = hi
        return out

    def forward(self, x):
        with M._Mode(self):
            s = M.nchw(M.conv_bn_act(self, self.conv1, self.bn1, x, *M.act_of(self.hs1)))
        out = OrderedDict()
        for i, blocks in enumerate(self.stages()):
            for b in blocks:
                s = b(s)
            out[i + 1] = s
        return out


class RetinaFace_Small(HipModule):
    """The JABD head (ECA -> FPN + NLM -> ECA -> SSH -> heads, as RetinaFace
    above) on a MobileNetV3_Small body: BASELINE config 1's "MobileNetV3-small
    + ECA head" (cfg_mnv3_small).  Lateral widths 24/48/96; ECA blocks
    eca_24 / eca_48 / eca_96 and eca_fpn."""
    eca_names = ("eca_24", "eca_48", "eca_96")

    def __init__(self, cfg=None, pretrained=False, mode="train"):
        super().__init__()
        if pretrained:
            raise RuntimeError("no pretrained MobileNetV3_Small checkpoint is shipped")
        self.body = MobileNetV3SmallBody(MobileNetV3_Small())
        oc = cfg["out_channel"]
        self.fpn = FPN([24, 48, 96], oc)
        self.ssh1 = SSH(oc, oc)
        self.ssh2 = SSH(oc, oc)
        self.ssh3 = SSH(oc, oc)
        self.ClassHead = nn.ModuleList([ClassHead(oc, 2) for _ in range(3)])
        self.BboxHead = nn.ModuleList([BboxHead(oc, 2) for _ in range(3)])
        self.LandmarkHead = nn.ModuleList([LandmarkHead(oc, 2) for _ in range(3)])
        self.eca_24 = eca_block(24)
        self.eca_48 = eca_block(48)
        self.eca_96 = eca_block(96)
        self.eca_fpn = eca_block(oc)
        self.mode = mode
        self.cfg = cfg

    def forward(self, inputs):
        return retinaface_forward(self, "mnv3", inputs)
