"""MobileNetV3-Large-ECA backbone modules — parameter-compatible with
nets/mobilenetV3.py:18-150,332-522 of the reference.

These modules hold the parameters (state_dict keys identical to the
reference); the detector forward runs through `RetinaFace.forward`'s fused
HIP plan (jabd_amd/engine.py), which reads them.  `SeModule` is built but —
as in the reference's Block_eca.forward (:140-150) — never applied.
"""
import math

import torch.nn as nn
from torch.nn import init


class SeModule(nn.Module):
    def __init__(self, in_size, reduction=4):
        super().__init__()
        mid = max(in_size // reduction, 8)
        self.se = nn.Sequential(
            nn.AdaptiveAvgPool2d(1),
            nn.Conv2d(in_size, mid, kernel_size=1, bias=False),
            nn.BatchNorm2d(mid),
            nn.ReLU(inplace=True),
            nn.Conv2d(mid, in_size, kernel_size=1, bias=False),
            nn.Hardsigmoid(),
        )


def eca_kernel_size(channel, b=1, gamma=2):
    k = int(abs((math.log(channel, 2) + b) / gamma))
    return k if k % 2 else k + 1


class eca_block(nn.Module):
    """In-block ECA (Hardsigmoid gate) — reference nets/mobilenetV3.py:332-348."""
    gate = "hsigmoid"

    def __init__(self, channel, b=1, gamma=2):
        super().__init__()
        k = eca_kernel_size(channel, b, gamma)
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.conv = nn.Conv1d(1, 1, kernel_size=k, padding=(k - 1) // 2, bias=False)
        self.sigmoid = nn.Sigmoid()
        self.Hsigmoid = nn.Hardsigmoid()


class Block_eca(nn.Module):
    """expand 1x1 -> depthwise kxk -> ECA -> project 1x1 (+skip) -> act."""

    def __init__(self, kernel_size, in_size, expand_size, out_size, act, se, stride):
        super().__init__()
        self.stride = stride
        self.kernel_size = kernel_size
        self.in_size, self.expand_size, self.out_size = in_size, expand_size, out_size
        self.act_name = "relu" if act is nn.ReLU else "hswish"
        self.conv1 = nn.Conv2d(in_size, expand_size, kernel_size=1, bias=False)
        self.bn1 = nn.BatchNorm2d(expand_size)
        self.act1 = act(inplace=True)
        self.conv2 = nn.Conv2d(expand_size, expand_size, kernel_size=kernel_size, stride=stride,
                               padding=kernel_size // 2, groups=expand_size, bias=False)
        self.bn2 = nn.BatchNorm2d(expand_size)
        self.act2 = act(inplace=True)
        self.se = SeModule(expand_size) if se else nn.Identity()
        self.eca = eca_block(expand_size)
        self.conv3 = nn.Conv2d(expand_size, out_size, kernel_size=1, bias=False)
        self.bn3 = nn.BatchNorm2d(out_size)
        self.act3 = act(inplace=True)
        self.skip = None
        if stride == 1 and in_size != out_size:
            self.skip = nn.Sequential(nn.Conv2d(in_size, out_size, kernel_size=1, bias=False),
                                      nn.BatchNorm2d(out_size))
        if stride == 2 and in_size != out_size:
            self.skip = nn.Sequential(
                nn.Conv2d(in_size, in_size, kernel_size=3, groups=in_size, stride=2, padding=1,
                          bias=False),
                nn.BatchNorm2d(in_size),
                nn.Conv2d(in_size, out_size, kernel_size=1, bias=True),
                nn.BatchNorm2d(out_size))
        if stride == 2 and in_size == out_size:
            self.skip = nn.Sequential(
                nn.Conv2d(in_size, out_size, kernel_size=3, groups=in_size, stride=2, padding=1,
                          bias=False),
                nn.BatchNorm2d(out_size))


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


# (kernel, in, expand, out, act, se, stride) per layer — reference :459-481
LARGE_ECA_LAYERS = (
    ((3, 16, 16, 16, nn.ReLU, False, 1), (3, 16, 64, 24, nn.ReLU, False, 2),
     (3, 24, 72, 24, nn.ReLU, False, 1), (5, 24, 72, 40, nn.ReLU, True, 2),
     (5, 40, 120, 40, nn.ReLU, True, 1), (5, 40, 120, 40, nn.ReLU, True, 1)),
    ((3, 40, 240, 80, nn.Hardswish, False, 2), (3, 80, 200, 80, nn.Hardswish, False, 1),
     (3, 80, 184, 80, nn.Hardswish, False, 1), (3, 80, 184, 80, nn.Hardswish, False, 1)),
    ((3, 80, 480, 112, nn.Hardswish, True, 1), (3, 112, 672, 112, nn.Hardswish, True, 1),
     (5, 112, 672, 160, nn.Hardswish, True, 2), (5, 160, 672, 160, nn.Hardswish, True, 1),
     (5, 160, 960, 160, nn.Hardswish, True, 1)),
)


class MobileNetV3_Large_eca(nn.Module):
    """Reference nets/mobilenetV3.py:452-522 (classifier tail kept for keys)."""

    def __init__(self, num_classes=1000, act=nn.Hardswish):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 16, kernel_size=3, stride=2, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(16)
        self.hs1 = act(inplace=True)
        for li, specs in enumerate(LARGE_ECA_LAYERS):
            blocks = [Block_eca(k, i, e, o, (a if a is nn.ReLU else act), se, s)
                      for (k, i, e, o, a, se, s) in specs]
            setattr(self, f"layer{li + 1}", nn.Sequential(*blocks))
        self.conv2 = nn.Conv2d(160, 960, kernel_size=1, stride=1, padding=0, bias=False)
        self.bn2 = nn.BatchNorm2d(960)
        self.hs2 = act(inplace=True)
        self.gap = nn.AdaptiveAvgPool2d(1)
        self.linear3 = nn.Linear(960, 1280, bias=False)
        self.bn3 = nn.BatchNorm1d(1280)
        self.hs3 = act(inplace=True)
        self.drop = nn.Dropout(0.2)
        self.linear4 = nn.Linear(1280, num_classes)
        _init_params(self)

    def forward(self, x):
        raise NotImplementedError("the JABD HIP path runs the backbone inside RetinaFace.forward")
