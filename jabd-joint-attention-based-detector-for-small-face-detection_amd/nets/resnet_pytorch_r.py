"""ResNets with torchvision's module layout and state_dict keys — the backbone
`models.resnet50()` of the reference's R50 detector
(nets/retinaface_eca_nonlocal.py:252; vendored copy nets/resnet_pytorch_r.py:27-390).

Every module runs libjabd kernels: Bottleneck/BasicBlock forwards are one
fused block each (eval: BN folded, downsample K-concatenated into the last
GEMM; training: the autograd graph of jabd_amd/train.py), ResNet.forward
runs the stem, the four stages, the pool and the classifier.  Pretrained
downloads are unavailable offline and raise."""
import torch
import torch.nn as nn

from jabd_amd import modules as M
from jabd_amd import train as T
from jabd_amd.engine import _R50Block
from jabd_amd.hipmodule import HipModule


def conv3x3(in_planes, out_planes, stride=1, groups=1, dilation=1):
    return M.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=dilation,
                    groups=groups, bias=False, dilation=dilation)


def conv1x1(in_planes, out_planes, stride=1):
    return M.Conv2d(in_planes, out_planes, kernel_size=1, stride=stride, bias=False)


def _check_plain(groups, base_width, dilation):
    if groups != 1 or base_width != 64 or dilation != 1:
        raise NotImplementedError("grouped / widened / dilated ResNet blocks are not built on "
                                  "the HIP path (JABD uses plain ResNets)")


class BasicBlock(HipModule):
    """conv3x3-BN-ReLU-conv3x3-BN (+identity) -ReLU (reference :38-84)."""
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64,
                 dilation=1, norm_layer=None):
        super().__init__()
        _check_plain(groups, base_width, dilation)
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = M.BatchNorm2d(planes)
        self.relu = M.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = M.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        xh = M.nhwc(x, "BasicBlock input").contiguous()
        with M._Mode(self):
            t = M.conv_bn_act(self, self.conv1, self.bn1, x, "relu")
            if self.downsample is not None:
                idn = M.nhwc(self.downsample(x)).contiguous()
            else:
                idn = xh
            if self.training:
                y = M.bn_nhwc(self.bn2, M.conv_nhwc(self.conv2, t), "relu", res=idn)
            else:
                from jabd_amd import functional as F
                pk = self._jabd_cached(x.device, lambda: F.pack_conv(self.conv2, self.bn2),
                                       tag="conv2")
                y = F.conv(t, pk, pad=1, act="relu", res=idn)
        return M.nchw(y)


class Bottleneck(HipModule):
    """1x1-3x3-1x1 bottleneck, stride on the 3x3 (v1.5), reference :87-143."""
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64,
                 dilation=1, norm_layer=None):
        super().__init__()
        _check_plain(groups, base_width, dilation)
        self.conv1 = conv1x1(inplanes, planes)
        self.bn1 = M.BatchNorm2d(planes)
        self.conv2 = conv3x3(planes, planes, stride)
        self.bn2 = M.BatchNorm2d(planes)
        self.conv3 = conv1x1(planes, planes * self.expansion)
        self.bn3 = M.BatchNorm2d(planes * self.expansion)
        self.relu = M.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        xh = M.nhwc(x, "Bottleneck input").contiguous()
        if self.training:
            return M.nchw(T._r50_block(self, xh))
        blk = self._jabd_cached(x.device, lambda: _R50Block(self))
        with torch.no_grad():
            return M.nchw(blk.forward(xh))


class ResNet(HipModule):
    def __init__(self, block=None, layers=(3, 4, 6, 3), num_classes=1000,
                 zero_init_residual=False, groups=1, width_per_group=64,
                 replace_stride_with_dilation=None, norm_layer=None):
        super().__init__()
        if block is None:
            block = Bottleneck
        if isinstance(block, (list, tuple)):  # ResNet(layers) as this module's r01 signature
            block, layers = Bottleneck, block
        _check_plain(groups, width_per_group, 1)
        if replace_stride_with_dilation not in (None, [False] * 3, (False,) * 3):
            raise NotImplementedError("dilated ResNet stages are not built on the HIP path")
        self.inplanes = 64
        self.dilation = 1
        self.groups = groups
        self.base_width = width_per_group
        self.conv1 = M.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = M.BatchNorm2d(64)
        self.relu = M.ReLU(inplace=True)
        self.maxpool = M.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = M.AdaptiveAvgPool2d((1, 1))
        self.fc = M.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.constant_(m.bn3.weight, 0)
                elif isinstance(m, BasicBlock):
                    nn.init.constant_(m.bn2.weight, 0)

    def _make_layer(self, block, planes, blocks, stride=1, dilate=False):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = M.ConvBNAct(conv1x1(self.inplanes, planes * block.expansion, stride),
                                     M.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def _forward_impl(self, x):
        with M._Mode(self):
            x = M.nchw(M.conv_bn_act(self, self.conv1, self.bn1, x, "relu"))
        x = self.maxpool(x)
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        with M._Mode(self):
            x = M.global_avg_pool(M.nhwc(x).contiguous())
        return self.fc(x)

    def forward(self, x):
        return self._forward_impl(x)


def _resnet(arch, block, layers, pretrained, progress, **kwargs):
    if pretrained:
        raise RuntimeError(f"pretrained {arch} weights need a download; this image is offline")
    return ResNet(block, layers, **kwargs)


def resnet18(pretrained=False, progress=True, **kwargs):
    return _resnet("resnet18", BasicBlock, [2, 2, 2, 2], pretrained, progress, **kwargs)


def resnet34(pretrained=False, progress=True, **kwargs):
    return _resnet("resnet34", BasicBlock, [3, 4, 6, 3], pretrained, progress, **kwargs)


def resnet50(pretrained=False, progress=True, **kwargs):
    return _resnet("resnet50", Bottleneck, [3, 4, 6, 3], pretrained, progress, **kwargs)


def resnet101(pretrained=False, progress=True, **kwargs):
    return _resnet("resnet101", Bottleneck, [3, 4, 23, 3], pretrained, progress, **kwargs)


def resnet152(pretrained=False, progress=True, **kwargs):
    return _resnet("resnet152", Bottleneck, [3, 8, 36, 3], pretrained, progress, **kwargs)


def resnet50_self(pretrained=False, progress=True, **kwargs):
    # the reference passes five stage counts; ResNet builds the first four (:304-314)
    return _resnet("resnet50", Bottleneck, [3, 4, 3, 3, 3], pretrained, progress, **kwargs)


def resnet101_self(pretrained=False, progress=True, **kwargs):
    return _resnet("resnet101", Bottleneck, [3, 4, 11, 12, 3], pretrained, progress, **kwargs)


def resnet152_self(pretrained=False, progress=True, **kwargs):
    return _resnet("resnet152", Bottleneck, [3, 8, 18, 18, 3], pretrained, progress, **kwargs)


def _grouped(name):
    def build(pretrained=False, progress=True, **kwargs):
        raise NotImplementedError(f"{name}: grouped/wide ResNets are not part of the JABD path")
    build.__name__ = name
    return build


resnext50_32x4d = _grouped("resnext50_32x4d")
resnext101_32x8d = _grouped("resnext101_32x8d")
wide_resnet50_2 = _grouped("wide_resnet50_2")
wide_resnet101_2 = _grouped("wide_resnet101_2")
