"""The module-level HIP path: the reference's nn.Modules run one by one.

RetinaFace.forward runs the whole detector as one fused plan (engine.py /
train.py).  But the reference's training scripts also build detectors inline
(train_mobilenetV3_ecagai.py:319-435, train_50_3_r.py:145-244) out of the
modules this package exports, and torchvision's IntermediateLayerGetter calls
a backbone's children one after another.  Every exported module therefore has
a forward of its own that runs libjabd kernels:

  leaf modules   Conv2d, BatchNorm2d/1d, ReLU, LeakyReLU, Hardswish,
                 Hardsigmoid, Sigmoid, MaxPool2d, AdaptiveAvgPool2d, Linear —
                 subclasses of the torch classes (same names, same state_dict
                 keys, `isinstance(m, nn.Conv2d)` still holds)
  composites     conv+BN+act Sequentials, Block_eca, Bottleneck, SSH, FPN,
                 NLM, eca_block, heads (nets/*) — one fused call each, the
                 same kernels and packs the fused plan uses

Layout: module inputs/outputs are logically NCHW (as the reference) and
physically NHWC — channels_last tensors, whose .permute(0, 2, 3, 1) is the
contiguous NHWC tensor the kernels take — so a chain of modules converts
nothing.  A plain NCHW-contiguous input is converted once (a channels_last
copy); the network input of a stem conv is read as NCHW directly.

Modes: training mode builds the autograd graph of libjabd kernels
(train.py); eval mode is inference only (folded BN, no autograd history),
as in the fused plan.  There is no CPU path.
"""
import ctypes

import torch
import torch.nn as nn

from . import functional as F
from . import train as T
from ._lib import call
from .hipmodule import HipModule

ACT = F.ACT


def _st():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


# ----------------------------------------------------------------------------- layout
def nhwc(x, what="module input"):
    """Logical NCHW tensor -> contiguous NHWC view (zero-copy if channels_last)."""
    F._check(what, x)
    if x.dim() != 4:
        raise ValueError(f"{what}: expected [B, C, H, W], got {tuple(x.shape)}")
    if not x.is_contiguous(memory_format=torch.channels_last):
        x = x.contiguous(memory_format=torch.channels_last)
    return x.permute(0, 2, 3, 1)


def nchw(y):
    """NHWC tensor -> the logical NCHW (channels_last) view the caller sees."""
    return y.permute(0, 3, 1, 2)


def _dense(x):
    """x unchanged if its storage is dense in NCHW or channels_last order."""
    if x.is_contiguous() or (x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)):
        return x
    return x.contiguous()


def _match_layout(t, ref):
    if ref.is_contiguous():
        return t.contiguous()
    return t.contiguous(memory_format=torch.channels_last)


class _Mode:
    """Eval mode = inference only (no autograd history, like the fused plan)."""

    def __init__(self, module):
        self.nograd = not module.training

    def __enter__(self):
        self.ctx = torch.no_grad() if self.nograd else None
        if self.ctx is not None:
            self.ctx.__enter__()

    def __exit__(self, *exc):
        if self.ctx is not None:
            self.ctx.__exit__(*exc)


# ----------------------------------------------------------------------------- autograd
class ActFn(torch.autograd.Function):
    """Elementwise activation over dense storage (jabd_act_f32 / _bwd_f32)."""

    @staticmethod
    def forward(ctx, x, act, slope):
        x = _dense(x)
        y = torch.empty_like(x)
        call("jabd_act_f32", x.data_ptr(), x.numel(), ACT[act], float(slope), y.data_ptr(), _st())
        if act in ("relu", "leaky", "hswish", "hsigmoid"):
            F.tap("act", act, slope, x)
        ctx.save_for_backward(x)
        ctx.cfg = (act, slope)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        act, slope = ctx.cfg
        dy = _match_layout(dy, x)
        dx = torch.empty_like(x)
        call("jabd_act_bwd_f32", x.data_ptr(), dy.data_ptr(), x.numel(), ACT[act], float(slope),
             dx.data_ptr(), _st())
        return dx, None, None


def activation(x, act, slope=0.0):
    F._check(f"{act} input", x)
    return ActFn.apply(x, act, slope)


class AdaptivePoolFn(torch.autograd.Function):
    """cat over sizes of AdaptiveAvgPool2d((s, s)) of NHWC x -> [B, S, C]."""

    @staticmethod
    def forward(ctx, x, sizes):
        B, H, W, C = x.shape
        out = F.adaptive_pool(x, sizes)
        ctx.cfg = (tuple(sizes), B, H, W, C)
        return out

    @staticmethod
    def backward(ctx, dy):
        sizes, B, H, W, C = ctx.cfg
        dy = dy.contiguous()
        dx = torch.empty((B, H, W, C), dtype=torch.float32, device=dy.device)
        arr = (ctypes.c_int32 * len(sizes))(*sizes)
        call("jabd_adaptive_pool_bwd_f32", dy.data_ptr(), B, H, W, C, arr, len(sizes),
             dx.data_ptr(), _st())
        return dx, None


class EcaScaleFn(torch.autograd.Function):
    """x * gate(Conv1d(mean_hw(x))) — eca_block.forward (nets/retinaface_r.py:219-224,
    nets/mobilenetV3.py:343-348) on NHWC x; gate 'sigmoid' or 'hsigmoid'."""

    @staticmethod
    def forward(ctx, x, w1d, gate):
        B, H, W, C = x.shape
        w1 = w1d.detach().reshape(-1).float().contiguous()
        scale, mean = F.eca_gate(F.channel_sums(x), H * W, w1, gate, return_mean=True)
        if gate == "hsigmoid":
            F.tap("eca", gate, mean, w1)
        y = torch.empty_like(x)
        call("jabd_channel_scale_f32", x.data_ptr(), B, H * W, C, scale.data_ptr(), y.data_ptr(),
             _st())
        ctx.save_for_backward(x, w1d, scale, mean)
        ctx.gate = gate
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w1d, scale, mean = ctx.saved_tensors
        dy = dy.contiguous()
        B, H, W, C = x.shape
        w1 = w1d.detach().reshape(-1).float().contiguous()
        k = w1.numel()
        HW = H * W
        nblk = max(1, min(64, HW // 256))
        part = torch.empty((B, nblk, C), dtype=torch.float32, device=x.device)
        dmean = torch.empty((B, C), dtype=torch.float32, device=x.device)
        dw1_img = torch.empty((B, k), dtype=torch.float32, device=x.device)
        dx = torch.empty_like(x)
        dw1 = torch.empty(k, dtype=torch.float32, device=x.device)
        call("jabd_eca_bwd_f32", dy.data_ptr(), x.data_ptr(), B, HW, C, scale.data_ptr(),
             mean.data_ptr(), w1.data_ptr(), k, ACT[ctx.gate], part.data_ptr(), nblk,
             dmean.data_ptr(), dw1_img.data_ptr(), dx.data_ptr(), dw1.data_ptr(), _st())
        return dx, dw1.view_as(w1d), None


class ScaleFn(torch.autograd.Function):
    """y = x * s[b][c] with s an input of its own (SeModule, nets/mobilenetV3.py:31-32)."""

    @staticmethod
    def forward(ctx, x, s):
        B, H, W, C = x.shape
        ctx.s_shape = s.shape
        s = s.reshape(B, C).contiguous()
        y = torch.empty_like(x)
        call("jabd_channel_scale_f32", x.data_ptr(), B, H * W, C, s.data_ptr(), y.data_ptr(),
             _st())
        ctx.save_for_backward(x, s)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, s = ctx.saved_tensors
        dy = dy.contiguous()
        B, H, W, C = x.shape
        nblk = max(1, min(64, (H * W) // 256))
        part = torch.empty((B, nblk, C), dtype=torch.float32, device=x.device)
        dx = torch.empty_like(x)
        call("jabd_scale_bwd_f32", dy.data_ptr(), x.data_ptr(), B, H * W, C, s.data_ptr(),
             part.data_ptr(), nblk, dx.data_ptr(), _st())
        return dx, part.sum(1).view(ctx.s_shape)


# ----------------------------------------------------------------------------- NHWC ops
def _geom(conv):
    if conv.dilation not in ((1, 1), 1) or conv.padding_mode != "zeros":
        raise NotImplementedError(f"{type(conv).__name__}: dilation / padding_mode "
                                  f"{conv.dilation} {conv.padding_mode} not supported on HIP")
    kh, kw = conv.kernel_size
    sh, sw = conv.stride
    ph, pw = conv.padding if isinstance(conv.padding, tuple) else (None, None)
    if kh != kw or sh != sw or ph != pw or ph is None:
        raise NotImplementedError(f"{type(conv).__name__}: square kernels/strides/paddings only")
    return kh, sh, ph


def conv_nhwc(conv, xh, nchw_in=False):
    """nn.Conv2d (dense or depthwise) on NHWC xh (or NCHW when nchw_in) -> NHWC."""
    k, stride, pad = _geom(conv)
    cin = conv.in_channels
    if conv.groups == 1:
        return T.ConvFn.apply(xh, conv.weight, conv.bias, stride, pad, nchw_in)
    if conv.groups == cin == conv.out_channels and conv.bias is None and pad == k // 2:
        if nchw_in:
            raise NotImplementedError("depthwise conv on an NCHW network input")
        return T.DwConvFn.apply(xh.contiguous(), conv.weight, stride)
    raise NotImplementedError(f"Conv2d groups={conv.groups} (only dense and depthwise k//2 "
                              "padding without bias are built)")


def bn_nhwc(bn, xh, act="none", slope=0.0, res=None):
    """nn.BatchNorm2d/1d (+ act, + residual before the act) on NHWC rows."""
    if bn.weight is None or bn.momentum is None:
        raise NotImplementedError("BatchNorm without affine / with momentum=None")
    C = xh.shape[-1]
    if bn.training or not bn.track_running_stats:
        if C % 4:
            raise NotImplementedError(f"training-mode BatchNorm over {C} channels (C % 4 != 0) "
                                      "outside a fused module")
        return T.bn_act(xh.contiguous(), bn, act, slope, res=res)
    if res is not None:
        raise NotImplementedError("eval BatchNorm with a residual")
    x = xh.contiguous()
    y = torch.empty_like(x)
    call("jabd_bn_eval_f32", x.data_ptr(), x.numel() // C, C, bn.running_mean.data_ptr(),
         bn.running_var.data_ptr(), float(bn.eps), bn.weight.data_ptr(), bn.bias.data_ptr(),
         ACT[act], float(slope), y.data_ptr(), _st())
    return y


def _is_nchw_input(x, conv):
    return conv.in_channels <= 4 and conv.groups == 1 and x.is_contiguous() and \
        not x.is_contiguous(memory_format=torch.channels_last)


def conv_bn_act(owner, conv, bn, x, act="none", slope=0.0):
    """conv -> BN -> act on a logical NCHW x (the reference's conv_bn Sequentials,
    a backbone stem); returns the NHWC result.  Eval: one fused launch with the
    BN folded into the packed weights (cached on `owner`)."""
    F._check("conv input", x)
    nchw_in = _is_nchw_input(x, conv)
    xin = x if nchw_in else nhwc(x)
    k, stride, pad = _geom(conv)
    if owner.training:
        return bn_nhwc(bn, conv_nhwc(conv, xin, nchw_in), act, slope)
    if conv.groups != 1:
        dev = x.device
        w, b = owner._jabd_cached(dev, lambda: F.pack_dw(conv, bn), tag="dw")
        y, _ = F.dwconv(xin.contiguous(), w, b, k, stride, act=act, slope=slope)
        return y
    if nchw_in and k == 3 and stride == 2 and pad == 1 and conv.in_channels == 3 and \
            conv.out_channels == 16 and act in ("hswish", "relu", "none") and conv.bias is None:
        w, b = owner._jabd_cached(x.device, lambda: _stem_pack(conv, bn), tag="stem")
        return F.stem(x, w, b, act)
    pk = owner._jabd_cached(x.device, lambda: F.pack_conv(conv, bn))
    return F.conv(xin, pk, stride=stride, pad=pad, act=act, slope=slope, nchw_in=nchw_in)


def _stem_pack(conv, bn):
    s, t = F.bn_fold(bn)
    return ((F.conv_weight_2d(conv.weight.detach().float()) * s[None, :]).contiguous(),
            t.detach().contiguous())


_ACT_OF = {}


def act_of(module):
    """(kind, slope) of an activation module (or None)."""
    for cls, fn in _ACT_OF.items():
        if isinstance(module, cls):
            return fn(module)
    return None


# ----------------------------------------------------------------------------- leaf modules
class Conv2d(HipModule, nn.Conv2d):
    def forward(self, x):
        with _Mode(self):
            F._check("Conv2d input", x)
            if _is_nchw_input(x, self):
                return nchw(conv_nhwc(self, x, nchw_in=True))
            return nchw(conv_nhwc(self, nhwc(x)))


class BatchNorm2d(HipModule, nn.BatchNorm2d):
    def forward(self, x):
        with _Mode(self):
            return nchw(bn_nhwc(self, nhwc(x)))


class BatchNorm1d(HipModule, nn.BatchNorm1d):
    def forward(self, x):
        with _Mode(self):
            F._check("BatchNorm1d input", x)
            if x.dim() != 2:
                raise NotImplementedError("BatchNorm1d over [B, C] only")
            B, C = x.shape
            return bn_nhwc(self, x.contiguous().view(B, 1, 1, C)).view(B, C)


class ReLU(HipModule, nn.ReLU):
    def forward(self, x):
        with _Mode(self):
            return activation(x, "relu")


class LeakyReLU(HipModule, nn.LeakyReLU):
    def forward(self, x):
        with _Mode(self):
            return activation(x, "leaky", self.negative_slope)


class Hardswish(HipModule, nn.Hardswish):
    def forward(self, x):
        with _Mode(self):
            return activation(x, "hswish")


class Hardsigmoid(HipModule, nn.Hardsigmoid):
    def forward(self, x):
        with _Mode(self):
            return activation(x, "hsigmoid")


class Sigmoid(HipModule, nn.Sigmoid):
    def forward(self, x):
        with _Mode(self):
            return activation(x, "sigmoid")


_ACT_OF.update({nn.ReLU: lambda m: ("relu", 0.0),
                nn.LeakyReLU: lambda m: ("leaky", m.negative_slope),
                nn.Hardswish: lambda m: ("hswish", 0.0)})


class MaxPool2d(HipModule, nn.MaxPool2d):
    def forward(self, x):
        with _Mode(self):
            k = self.kernel_size if isinstance(self.kernel_size, int) else self.kernel_size[0]
            s = self.stride if isinstance(self.stride, int) else self.stride[0]
            p = self.padding if isinstance(self.padding, int) else self.padding[0]
            if (k, s, p) != (3, 2, 1) or self.ceil_mode or self.dilation not in (1, (1, 1)):
                raise NotImplementedError("MaxPool2d(3, 2, 1) (the ResNet stem pool) only")
            return nchw(T.MaxPoolFn.apply(nhwc(x).contiguous()))


def _square(size):
    if isinstance(size, int):
        return size
    if len(size) == 2 and size[0] == size[1] and size[0] is not None:
        return size[0]
    raise NotImplementedError(f"AdaptiveAvgPool2d output {size}: square sizes only")


class AdaptiveAvgPool2d(HipModule, nn.AdaptiveAvgPool2d):
    def forward(self, x):
        with _Mode(self):
            s = _square(self.output_size)
            xh = nhwc(x)
            B, _, _, C = xh.shape
            out = AdaptivePoolFn.apply(xh, (s,))
            return nchw(out.view(B, s, s, C))


class Linear(HipModule, nn.Linear):
    """x [B, K] @ W^T + b as a 1x1 conv over a 1x1 map (MFMA GEMM)."""

    def forward(self, x):
        with _Mode(self):
            F._check("Linear input", x)
            if x.dim() != 2:
                raise NotImplementedError("Linear over [B, K] only")
            B, K = x.shape
            N = self.out_features
            y = T.ConvFn.apply(x.contiguous().view(B, 1, 1, K), self.weight.view(N, K, 1, 1),
                               self.bias, 1, 0, False)
            return y.view(B, N)


def global_avg_pool(xh):
    """AdaptiveAvgPool2d(1) + flatten of NHWC xh -> [B, C]."""
    B, _, _, C = xh.shape
    return AdaptivePoolFn.apply(xh, (1,)).view(B, C)


# ----------------------------------------------------------------------------- sequentials
def run_sequential(seq, x):
    """Run nn.Sequential-like children with the conv -> BN -> act peephole fused
    (torchvision's IntermediateLayerGetter walks a backbone's children this way)."""
    mods = list(seq)
    i = 0
    while i < len(mods):
        m = mods[i]
        if isinstance(m, nn.Conv2d) and i + 1 < len(mods) and isinstance(mods[i + 1],
                                                                         nn.BatchNorm2d):
            a = act_of(mods[i + 2]) if i + 2 < len(mods) else None
            n = 3 if a is not None else 2
            with _Mode(m):
                x = nchw(conv_bn_act(m, m, mods[i + 1], x, *(a or ("none", 0.0))))
            i += n
            continue
        x = m(x)
        i += 1
    return x


class FusedSequential(HipModule, nn.Sequential):
    """nn.Sequential whose conv -> BN -> act runs are fused (keys unchanged):
    the reference's conv_bn / conv_bn1X1 / conv_bn_no_relu / conv_dw pieces."""

    def forward(self, x):
        return run_sequential(self, x)


ConvBNAct = FusedSequential


# ----------------------------------------------------------------------------- gates
def se_scale_eval(se, dh, owner):
    """SeModule gate hsigmoid(conv(relu(bn(conv(GAP(d)))))) -> [B, C] (eval)."""
    seq = se.se
    B, _, _, C = dh.shape
    p1, p2 = owner._jabd_cached(dh.device, lambda: (F.pack_conv(seq[1], seq[2]),
                                                    F.pack_conv(seq[4])), tag="se")
    g = global_avg_pool(dh).view(B, 1, 1, C)
    t = F.conv(g, p1, act="relu")
    return F.conv(t, p2, act="hsigmoid").view(B, C)


def se_scale_train(se, dh):
    """SeModule gate in training mode -> [B, 1, 1, C] (BN over the batch's 1x1
    maps; a hidden width that is not a multiple of 4 is zero-padded)."""
    seq = se.se
    B, _, _, C = dh.shape
    g = global_avg_pool(dh).view(B, 1, 1, C)
    mid = seq[1].out_channels
    mp = (mid + 3) // 4 * 4
    t = T.ConvFn.apply(g, T._padw(seq[1].weight, cout=mp), None, 1, 0, False)
    t = T.bn_act(t, seq[2], "relu")
    t = T.ConvFn.apply(t, T._padw(seq[4].weight, cin=mp), None, 1, 0, False)
    return ActFn.apply(t, "hsigmoid", 0.0)


def beca_gate(xh, w1d):
    """BECA gate hardsigmoid(conv1d(std_hw(x))) -> [B, C] without applying it
    (eval: the consumer conv scales its operand on load)."""
    B, H, W, C = xh.shape
    w = w1d.detach().reshape(-1).float().contiguous()
    stats = torch.empty((4, B * C), dtype=torch.float32, device=xh.device)
    from .ops import beca_part
    part = beca_part(B, H * W, C, xh.device)
    call("jabd_beca_fwd_f32", xh.data_ptr(), B, H * W, C, w.data_ptr(), w.numel(), None,
         stats.data_ptr(), part.data_ptr(), part.numel(), _st())
    return stats[3].view(B, C)
