"""MobileNetV1-0.25 — drop-in for the reference nets/mobilenet025.py:1-64 (the
mobilenet0.25 backbone train_50_3_r.py:152-162 builds under
IntermediateLayerGetter).  Stages are fused conv+BN+LeakyReLU Sequentials
(depthwise and pointwise) over libjabd kernels."""
from jabd_amd import modules as M
from jabd_amd.hipmodule import HipModule
from nets.mobilenetV3 import conv_bn, conv_dw
import torch.nn as nn


class MobileNetV1(HipModule):
    def __init__(self):
        super().__init__()
        self.stage1 = nn.Sequential(conv_bn(3, 8, 2, leaky=0.1), conv_dw(8, 16, 1),
                                    conv_dw(16, 32, 2), conv_dw(32, 32, 1),
                                    conv_dw(32, 64, 2), conv_dw(64, 64, 1))
        self.stage2 = nn.Sequential(conv_dw(64, 128, 2), *[conv_dw(128, 128, 1) for _ in range(5)])
        self.stage3 = nn.Sequential(conv_dw(128, 256, 2), conv_dw(256, 256, 1))
        self.avg = M.AdaptiveAvgPool2d((1, 1))
        self.fc = M.Linear(256, 1000)

    def forward(self, x):
        x = self.stage3(self.stage2(self.stage1(x)))
        with M._Mode(self):
            x = M.global_avg_pool(M.nhwc(x).contiguous())
        return self.fc(x)
