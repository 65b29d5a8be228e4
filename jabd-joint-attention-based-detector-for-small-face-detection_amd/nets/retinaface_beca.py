"""JABD-MobileNetV3-BECA RetinaFace — the detector that
train_mobilenetV3_ecagai.py:39-435 defines inline (inside its __main__), as an
importable module with the same class names, constructor signatures and
state_dict keys, so a checkpoint of that script loads here:

  * eca_block  — BECA: per-channel standard deviation over H*W -> Conv1d ->
                 Hardsigmoid -> x*y (:286-316)
  * NLM        — ch=40, PSP sizes (1, 3, 6, 8) -> S = 110 pooled rows (:161-234)
  * FPN        — bicubic align_corners up-sampling, then the shared NLM(40),
                 then the lateral add (:237-285)
  * RetinaFace — MobileNetV3_Large_eca body, BECA on C3/C4/C5 and on every
                 FPN level, SSH, 1x1 heads (:319-435); cfg_mnet only (the
                 script's 'Resnet50' / 'Resnet152' branches call torchvision
                 backbones; nets.retinaface_eca_nonlocal is the R50 detector)

RetinaFace.forward runs the fused HIP plan (engine.py, eval; train.py,
training) with the BECA gates applied on the consumer convs' operand load in
eval; every class also runs standalone on libjabd kernels.
"""
import math

import torch.nn as nn

from jabd_amd import modules as M
from jabd_amd.engine import retinaface_forward
from jabd_amd.hipmodule import HipModule
from jabd_amd.ops import BecaFn
from nets._getter import IntermediateLayerGetter
from nets.layers import SSH, conv_bn, conv_bn1X1, conv_bn_no_relu, fpn_forward  # noqa: F401
from nets.mobilenetV3 import MobileNetV3_Large_eca, mean_channels, stdv_channels  # noqa: F401
from nets.retinaface_r import NLM as _NLM
from nets.retinaface_r import BboxHead, ClassHead, LandmarkHead  # noqa: F401
from nets.retinaface_r import PSPModule as _PSP


class PSPModule(_PSP):
    """PSPModule with the script's default sizes (1, 3, 6, 8) (:161-180)."""

    def __init__(self, sizes=(1, 3, 6, 8), dimension=2):
        super().__init__(sizes, dimension)


class NLM(_NLM):
    """NLM(in_channels, scale=1, psp_size=(1, 3, 6, 8), ch=40) (:182-234):
    q/k/v 1x1 convs to ch=40, PSP-pooled keys/values, softmax attention,
    W (zero-initialised) back to in_channels, + x."""

    def __init__(self, in_channels, scale=1, psp_size=(1, 3, 6, 8), ch=40):
        super().__init__(in_channels, scale, psp_size, ch)


class FPN(HipModule):
    """Laterals, bicubic(align_corners) up-sample -> shared NLM(40) -> add,
    merges (:237-285)."""
    upsample_mode = "bicubic"

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
    """BECA (:297-316): x * Hardsigmoid(Conv1d(stdv_channels(x)))."""

    def __init__(self, channel, b=1, gamma=2):
        super().__init__()
        k = int(abs((math.log(channel, 2) + b) / gamma))
        k = k if k % 2 else k + 1
        self.avg_pool = M.AdaptiveAvgPool2d(1)
        self.conv = nn.Conv1d(1, 1, kernel_size=k, padding=(k - 1) // 2, bias=False)
        self.sigmoid = M.Sigmoid()
        self.Hsigmoid = M.Hardsigmoid()
        self.contrast = stdv_channels

    def forward(self, x):
        xh = M.nhwc(x, "eca_block input").contiguous()
        with M._Mode(self):
            return M.nchw(BecaFn.apply(xh, self.conv.weight.reshape(-1)))


class RetinaFace(HipModule):
    head_gate = "beca"

    def __init__(self, cfg=None, pretrained=False, mode="train"):
        super().__init__()
        if cfg["name"] != "mobilenet0.25":
            raise NotImplementedError(
                "the BECA script's 'Resnet50'/'Resnet152' branches wrap torchvision backbones; "
                "use nets.retinaface_eca_nonlocal.RetinaFace for the R50 detector")
        if pretrained:
            raise RuntimeError("the reference's pretrained backbone checkpoint is not shipped")
        backbone = MobileNetV3_Large_eca()
        self.body = IntermediateLayerGetter(backbone, cfg["return_layers"])
        c = cfg["in_channel"]
        oc = cfg["out_channel"]
        self.fpn = FPN([c * 2, c * 4, c * 8], oc)
        self.ssh1 = SSH(oc, oc)
        self.ssh2 = SSH(oc, oc)
        self.ssh3 = SSH(oc, oc)
        self.ClassHead = self._make_class_head(fpn_num=3, inchannels=oc)
        self.BboxHead = self._make_bbox_head(fpn_num=3, inchannels=oc)
        self.LandmarkHead = self._make_landmark_head(fpn_num=3, inchannels=oc)
        self.eca_40 = eca_block(40)
        self.eca_80 = eca_block(80)
        self.eca_160 = eca_block(160)
        self.eca_fpn = eca_block(40)
        self.mode = mode
        self.cfg = cfg

    def _make_class_head(self, fpn_num=3, inchannels=64, anchor_num=2):
        return nn.ModuleList([ClassHead(inchannels, anchor_num) for _ in range(fpn_num)])

    def _make_bbox_head(self, fpn_num=3, inchannels=64, anchor_num=2):
        return nn.ModuleList([BboxHead(inchannels, anchor_num) for _ in range(fpn_num)])

    def _make_landmark_head(self, fpn_num=3, inchannels=64, anchor_num=2):
        return nn.ModuleList([LandmarkHead(inchannels, anchor_num) for _ in range(fpn_num)])

    def forward(self, inputs):
        return retinaface_forward(self, "mnv3", inputs)
