"""SSH context module, the plain FPN and the conv helpers — drop-in for the
reference nets/layers.py:10-119 (same names, constructor signatures and
state_dict keys).  Every module's forward runs libjabd kernels
(jabd_amd/modules.py); inside RetinaFace.forward the same packs run as part
of the fused plan."""
import torch
import torch.nn as nn  # noqa: F401  (the reference module's namespace)

from jabd_amd import modules as M
from jabd_amd import train as T
from jabd_amd.engine import FPNPack, SSHPack
from jabd_amd.hipmodule import HipModule


def conv_bn(inp, oup, stride=1, leaky=0):
    """3x3 conv + BN + LeakyReLU (nets/layers.py:10-15)."""
    return M.ConvBNAct(M.Conv2d(inp, oup, 3, stride, 1, bias=False), M.BatchNorm2d(oup),
                       M.LeakyReLU(negative_slope=leaky, inplace=True))


def conv_bn1X1(inp, oup, stride, leaky=0):
    """1x1 conv + BN + LeakyReLU (nets/layers.py:17-22)."""
    return M.ConvBNAct(M.Conv2d(inp, oup, 1, stride, padding=0, bias=False), M.BatchNorm2d(oup),
                       M.LeakyReLU(negative_slope=leaky, inplace=True))


def conv_bn_no_relu(inp, oup, stride):
    """3x3 conv + BN (nets/layers.py:28-32)."""
    return M.ConvBNAct(M.Conv2d(inp, oup, 3, stride, 1, bias=False), M.BatchNorm2d(oup))


class SSH(HipModule):
    """3x3 (C/2) | 3x3->3x3 (C/4) | 3x3->3x3->3x3 (C/4), concat, ReLU
    (nets/layers.py:37-68)."""

    def __init__(self, in_channel, out_channel):
        super().__init__()
        assert out_channel % 4 == 0
        self.leaky = 0.1 if out_channel <= 64 else 0.0
        self.conv3X3 = conv_bn_no_relu(in_channel, out_channel // 2, stride=1)
        self.conv5X5_1 = conv_bn(in_channel, out_channel // 4, stride=1, leaky=self.leaky)
        self.conv5X5_2 = conv_bn_no_relu(out_channel // 4, out_channel // 4, stride=1)
        self.conv7X7_2 = conv_bn(out_channel // 4, out_channel // 4, stride=1, leaky=self.leaky)
        self.conv7x7_3 = conv_bn_no_relu(out_channel // 4, out_channel // 4, stride=1)

    def forward(self, inputs):
        xh = M.nhwc(inputs, "SSH input")
        if self.training:
            return M.nchw(T.ssh_train(self, xh))
        pk = self._jabd_cached(inputs.device, lambda: SSHPack(self))
        with torch.no_grad():
            return M.nchw(pk.forward(xh.contiguous()))


def fpn_forward(fpn, inputs, nlm):
    """FPN.forward for both FPN flavours: inputs = list of 3 logical-NCHW maps
    (or the IntermediateLayerGetter OrderedDict) -> [out1, out2, out3]."""
    if isinstance(inputs, dict):
        inputs = list(inputs.values())
    feats = [M.nhwc(t, "FPN input").contiguous() for t in inputs]
    if fpn.training:
        return [M.nchw(o) for o in T.fpn_train(fpn, feats, nlm)]
    pk = fpn._jabd_cached(feats[0].device, lambda: FPNPack(fpn, nlm))
    with torch.no_grad():
        return [M.nchw(o) for o in pk.forward(feats)]


class FPN(HipModule):
    """Plain FPN: 1x1 laterals, nearest up-sample + add, 3x3 merges
    (nets/layers.py:70-119; forward takes the backbone's OrderedDict)."""

    def __init__(self, in_channels_list, out_channels):
        super().__init__()
        self.leaky = 0.1 if out_channels <= 64 else 0.0
        self.output1 = conv_bn1X1(in_channels_list[0], out_channels, stride=1, leaky=self.leaky)
        self.output2 = conv_bn1X1(in_channels_list[1], out_channels, stride=1, leaky=self.leaky)
        self.output3 = conv_bn1X1(in_channels_list[2], out_channels, stride=1, leaky=self.leaky)
        self.merge1 = conv_bn(out_channels, out_channels, leaky=self.leaky)
        self.merge2 = conv_bn(out_channels, out_channels, leaky=self.leaky)

    def forward(self, inputs):
        return fpn_forward(self, inputs, None)


