"""RetinaFace-R50 + ECA + NLM — drop-in for the reference
nets/retinaface_eca_nonlocal.py:37-359 (the model predict.py loads).
Same names/keys (incl. the unused `Nlm` and `IouHead` modules).
RetinaFace.forward runs the fused HIP plan (jabd_amd/engine.py); the other
modules have HIP forwards of their own (jabd_amd/modules.py)."""
import torch.nn as nn

from jabd_amd import modules as M
from jabd_amd.engine import retinaface_forward
from jabd_amd.hipmodule import HipModule
from nets._getter import IntermediateLayerGetter
from nets.layers import SSH, conv_bn, conv_bn1X1, fpn_forward
from nets.resnet_pytorch_r import resnet50
from nets.retinaface_r import (BboxHead, ClassHead, LandmarkHead, NLM, PSPModule,  # noqa: F401
                               _Head1x1)
from nets.retinaface_r import eca_block as _eca_sigmoid


class FPN(HipModule):
    """Laterals, nearest up-sample -> shared NLM(256) -> add, merges (reference :37-90)."""

    def __init__(self, in_channels_list, out_channels):
        super().__init__()
        self.leaky = 0.1 if out_channels <= 64 else 0.0
        self.output1 = conv_bn1X1(in_channels_list[0], out_channels, stride=1, leaky=self.leaky)
        self.output2 = conv_bn1X1(in_channels_list[1], out_channels, stride=1, leaky=self.leaky)
        self.output3 = conv_bn1X1(in_channels_list[2], out_channels, stride=1, leaky=self.leaky)
        self.merge1 = conv_bn(out_channels, out_channels, leaky=self.leaky)
        self.merge2 = conv_bn(out_channels, out_channels, leaky=self.leaky)
        self.Nlm = NLM(256)

    def forward(self, inputs):
        return fpn_forward(self, inputs, self.Nlm)


class IOUHead(_Head1x1):
    k = 1

    def __init__(self, inchannels=512, num_anchors=2):
        super().__init__()
        self.conv1x1 = M.Conv2d(inchannels, num_anchors, kernel_size=(1, 1), stride=1, padding=0)


class eca_block(_eca_sigmoid):
    """Sigmoid-gated ECA (reference :203-219), same as nets/retinaface_r.py's."""


class RetinaFace(HipModule):
    def __init__(self, cfg=None, pretrained=False, mode="train"):
        super().__init__()
        if cfg["name"] != "Resnet50":
            raise ValueError("this drop-in implements the ResNet-50 JABD detector (cfg_re50)")
        backbone = resnet50(pretrained=pretrained)
        self.body = IntermediateLayerGetter(backbone, cfg["return_layers"])
        c = cfg["in_channel"]
        oc = cfg["out_channel"]
        self.fpn = FPN([c * 2, c * 4, c * 8], oc)
        self.ssh1 = SSH(oc, oc)
        self.ssh2 = SSH(oc, oc)
        self.ssh3 = SSH(oc, oc)
        self.ClassHead = nn.ModuleList([ClassHead(oc, 2) for _ in range(3)])
        self.BboxHead = nn.ModuleList([BboxHead(oc, 2) for _ in range(3)])
        self.LandmarkHead = nn.ModuleList([LandmarkHead(oc, 2) for _ in range(3)])
        self.IouHead = nn.ModuleList([BboxHead(oc, 2), BboxHead(oc, 2), IOUHead(oc, 2)])
        self.Nlm = NLM(256)
        self.eca_64 = eca_block(512)
        self.eca_128 = eca_block(1024)
        self.eca_256 = eca_block(2048)
        self.eca_fpn = eca_block(256)
        self.mode = mode
        self.cfg = cfg

    def forward(self, inputs):
        return retinaface_forward(self, "r50", inputs)
