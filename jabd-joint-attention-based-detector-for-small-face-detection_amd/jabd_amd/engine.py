"""Fused HIP forward plans for the two JABD detectors.

An Engine reads a RetinaFace module's parameters, folds eval-mode BatchNorm
into the convolutions, packs every weight into the MFMA fragment order once
(re-packed only when a parameter or buffer changes version), and runs the
forward as a fixed sequence of libjabd kernels on NHWC fp32 activations:

  MobileNetV3-JABD (nets/retinaface_r.py:304-343):
    stem conv3x3/s2 (reads the NCHW input directly) -> 15 x [expand GEMM ->
    depthwise (+ECA pool partials) -> ECA gate -> project GEMM with the ECA
    scale applied on load and the skip branch K-concatenated / added] ->
    head ECA -> FPN laterals -> NLM (fused with nearest up-sample and add) ->
    merge convs -> ECA -> SSH convs writing channel slices -> heads written
    straight into loc/conf/landm.
  RetinaFace-R50 (nets/retinaface_eca_nonlocal.py:314-359): 7x7 stem +
    maxpool, bottlenecks with the downsample folded into conv3's GEMM, then
    the same head.

There is no CPU path: inputs must be float32 tensors on the GPU.
"""
import os

import torch

from . import functional as F

NLM_SIZES_DEFAULT = (1, 4, 8, 12)
# MNv3 blocks run expand 1x1 + depthwise as one kernel (csrc/expdw.hip);
# JABD_FUSE_EXPAND_DW=0 selects the two-kernel path (A/B measurement, tests).
FUSE_EXPAND_DW = os.environ.get("JABD_FUSE_EXPAND_DW", "1") != "0"


def _params_signature(module):
    return tuple(t._version for t in module.parameters()) + tuple(
        t._version for t in module.buffers()) + tuple(
        t.data_ptr() for t in module.parameters())


def _w1d(eca):
    return eca.conv.weight.detach().reshape(-1).float().contiguous()


class _Head:
    """ECA -> FPN(+NLM) -> ECA -> SSH -> heads, shared by both detectors."""

    def __init__(self, m, eca_names, nlm):
        fpn = m.fpn
        self.leaky = fpn.leaky
        self.eca_in = [_w1d(getattr(m, n)) for n in eca_names]
        self.lat = [F.pack_conv(o[0], o[1]) for o in (fpn.output1, fpn.output2, fpn.output3)]
        self.merge1 = F.pack_conv(fpn.merge1[0], fpn.merge1[1])
        self.merge2 = F.pack_conv(fpn.merge2[0], fpn.merge2[1])
        self.nlm_sizes = tuple(nlm.psp.sizes)
        C, ch = nlm.in_channels, nlm.ch
        d = lambda t: t.detach().float().contiguous()  # noqa: E731
        self.nlm_w = (d(nlm.f_query.weight.view(ch, C)), d(nlm.f_query.bias),
                      d(nlm.f_key.weight.view(ch, C)), d(nlm.f_key.bias),
                      d(nlm.f_value.weight.view(ch, C)), d(nlm.f_value.bias),
                      d(nlm.W.weight.view(C, ch)), d(nlm.W.bias))
        self.eca_fpn = _w1d(m.eca_fpn)
        self.ssh = []
        q = m.ssh1.conv5X5_1[0].out_channels
        qp = (q + 3) // 4 * 4 if q % 4 else None  # 10-channel branches stored as 12
        # SSH (nets/layers.py:37-68): the two branches that read `o` (conv3X3,
        # conv5X5_1) and the two that read t (conv5X5_2, conv7X7_2) run as one
        # GEMM each with a split output (fused along N); every part's output
        # channels are padded to a multiple of 4 for the vector epilogue.
        q4 = (q + 3) // 4 * 4
        h2 = m.ssh1.conv3X3[0].out_channels
        # (R50's 256-channel SSH keeps five GEMMs: each takes the 32x32 k x k
        # kernel, which the split output does not)
        self.ssh_split = h2 % 4 == 0 and m.ssh1.conv3X3[0].in_channels % 32 != 0
        for s in (m.ssh1, m.ssh2, m.ssh3):
            if self.ssh_split:
                self.ssh.append((
                    F.pack_conv_cat([(s.conv3X3[0], s.conv3X3[1], None),
                                     (s.conv5X5_1[0], s.conv5X5_1[1], qp)]),
                    F.pack_conv_cat([(s.conv5X5_2[0], s.conv5X5_2[1], q4),
                                     (s.conv7X7_2[0], s.conv7X7_2[1], qp)], cin_pad=qp),
                    F.pack_conv(s.conv7x7_3[0], s.conv7x7_3[1], cin_pad=qp)))
                continue
            self.ssh.append((F.pack_conv(s.conv3X3[0], s.conv3X3[1]),
                             F.pack_conv(s.conv5X5_1[0], s.conv5X5_1[1], cout_pad=qp),
                             F.pack_conv(s.conv5X5_2[0], s.conv5X5_2[1], cin_pad=qp),
                             F.pack_conv(s.conv7X7_2[0], s.conv7X7_2[1], cin_pad=qp,
                                         cout_pad=qp),
                             F.pack_conv(s.conv7x7_3[0], s.conv7x7_3[1], cin_pad=qp)))
        self.heads = []
        for i in range(3):
            convs = (m.BboxHead[i].conv1x1, m.ClassHead[i].conv1x1, m.LandmarkHead[i].conv1x1)
            w = torch.cat([c.weight.detach().float().reshape(c.weight.shape[0], -1) for c in convs])
            b = torch.cat([c.bias.detach().float() for c in convs])
            self.heads.append((w.contiguous(), b.contiguous()))

    def forward(self, feats, softmax):
        B = feats[0].shape[0]
        lat = []
        for f, w1d, pk in zip(feats, self.eca_in, self.lat):
            hw = f.shape[1] * f.shape[2]
            sc = F.eca_gate(F.channel_sums(f), hw, w1d, "sigmoid")
            lat.append(F.conv(f, pk, act="leaky", slope=self.leaky, ascale=sc))
        o1, o2, o3 = lat
        m2 = F.nlm_fused(o3, o2, self.nlm_w, self.nlm_sizes)
        o2 = F.conv(m2, self.merge2, pad=1, act="leaky", slope=self.leaky)
        m1 = F.nlm_fused(o2, o1, self.nlm_w, self.nlm_sizes)
        o1 = F.conv(m1, self.merge1, pad=1, act="leaky", slope=self.leaky)
        levels = [o1, o2, o3]
        A = sum(2 * o.shape[1] * o.shape[2] for o in levels)
        dev = o1.device
        loc = torch.empty((B, A, 4), dtype=torch.float32, device=dev)
        conf = torch.empty((B, A, 2), dtype=torch.float32, device=dev)
        landm = torch.empty((B, A, 10), dtype=torch.float32, device=dev)
        a_off = 0
        for i, o in enumerate(levels):
            _, h, w, C = o.shape
            sc = F.eca_gate(F.channel_sums(o), h * w, self.eca_fpn, "sigmoid")
            feat = torch.empty((B, h, w, C), dtype=torch.float32, device=dev)
            if self.ssh_split:
                # feat = [conv3X3 (C/2) | conv5X5_2 (C/4) | conv7x7_3 (C/4)]; the
                # fused middle GEMM writes conv5X5_2 padded to a multiple of 4,
                # whose zero pad channels conv7x7_3 overwrites right after
                ca, cb, c73 = self.ssh[i]
                qp_ = cb.Cin
                t = torch.empty((B, h, w, qp_), dtype=torch.float32, device=dev)
                t2 = torch.empty((B, h, w, qp_), dtype=torch.float32, device=dev)
                F.conv(o, ca, pad=1, act="relu", ascale=sc, out=feat, out_c0=0, y2=t,
                       nsplit=C // 2, act2="leaky", slope2=self.leaky)
                F.conv(t, cb, pad=1, act="relu", out=feat, out_c0=C // 2, y2=t2,
                       nsplit=cb.Cout - qp_, act2="leaky", slope2=self.leaky)
                F.conv(t2, c73, pad=1, act="relu", out=feat, out_c0=3 * C // 4)
            else:
                c3, c51, c52, c72, c73 = self.ssh[i]
                F.conv(o, c3, pad=1, act="relu", ascale=sc, out=feat, out_c0=0)
                t = F.conv(o, c51, pad=1, act="leaky", slope=self.leaky, ascale=sc)
                F.conv(t, c52, pad=1, act="relu", out=feat, out_c0=C // 2)
                t2 = F.conv(t, c72, pad=1, act="leaky", slope=self.leaky)
                F.conv(t2, c73, pad=1, act="relu", out=feat, out_c0=3 * C // 4)
            wt, bs = self.heads[i]
            F.heads(feat, wt, bs, loc, conf, landm, a_off, softmax)
            a_off += 2 * h * w
        return loc, conf, landm


class _MNv3Block:
    def __init__(self, blk):
        self.k, self.stride, self.act = blk.kernel_size, blk.stride, blk.act_name
        self.expand = F.pack_conv(blk.conv1, blk.bn1)
        self.dw_w, self.dw_b = F.pack_dw(blk.conv2, blk.bn2)
        self.eca = _w1d(blk.eca)
        sk = blk.skip
        self.skip_dw = None
        if sk is None:
            self.kind = "identity"
            self.project = F.pack_conv(blk.conv3, blk.bn3)
        elif blk.stride == 1:
            self.kind = "concat"
            s, t = F.bn_fold(sk[1])
            w2 = F.conv_weight_2d(sk[0].weight.detach().float()) * s[None, :]
            self.project = F.pack_conv(blk.conv3, blk.bn3, extra=(w2, t))
        elif len(sk) == 4:
            self.kind = "dw_concat"
            self.skip_dw = F.pack_dw(sk[0], sk[1])
            s, t = F.bn_fold(sk[3], sk[2].bias.detach().float())
            w2 = F.conv_weight_2d(sk[2].weight.detach().float()) * s[None, :]
            self.project = F.pack_conv(blk.conv3, blk.bn3, extra=(w2, t))
        else:
            self.kind = "dw_residual"
            self.skip_dw = F.pack_dw(sk[0], sk[1])
            self.project = F.pack_conv(blk.conv3, blk.bn3)

    def forward(self, x):
        if FUSE_EXPAND_DW:
            d, part = F.expand_dw(x, self.expand, self.dw_w, self.dw_b, self.k, self.stride,
                                  act=self.act)
        else:
            e = F.conv(x, self.expand, act=self.act)
            d, part = F.dwconv(e, self.dw_w, self.dw_b, self.k, self.stride, act=self.act,
                               partials=True)
        sc = F.eca_gate(part, d.shape[1] * d.shape[2], self.eca, "hsigmoid")
        if self.kind == "identity":
            return F.conv(d, self.project, act=self.act, ascale=sc, res=x)
        if self.kind == "concat":
            return F.conv(d, self.project, act=self.act, ascale=sc, x2=x)
        t, _ = F.dwconv(x, self.skip_dw[0], self.skip_dw[1], 3, 2)
        if self.kind == "dw_concat":
            return F.conv(d, self.project, act=self.act, ascale=sc, x2=t)
        return F.conv(d, self.project, act=self.act, ascale=sc, res=t)


class _R50Block:
    def __init__(self, blk):
        self.stride = blk.stride
        self.c1 = F.pack_conv(blk.conv1, blk.bn1)
        self.c2 = F.pack_conv(blk.conv2, blk.bn2)
        if blk.downsample is not None:
            s, t = F.bn_fold(blk.downsample[1])
            w2 = F.conv_weight_2d(blk.downsample[0].weight.detach().float()) * s[None, :]
            self.c3 = F.pack_conv(blk.conv3, blk.bn3, extra=(w2, t))
            self.down = True
        else:
            self.c3 = F.pack_conv(blk.conv3, blk.bn3)
            self.down = False

    def forward(self, x):
        t = F.conv(x, self.c1, act="relu")
        t = F.conv(t, self.c2, stride=self.stride, pad=1, act="relu")
        if self.down:
            return F.conv(t, self.c3, act="relu", x2=x, x2_stride=self.stride)
        return F.conv(t, self.c3, act="relu", res=x)


class Engine:
    def __init__(self, model, kind):
        self.model, self.kind = model, kind
        self.sig = None

    def _refresh(self):
        m = self.model
        with torch.no_grad():
            if self.kind == "mnv3":
                s_, t_ = F.bn_fold(m.body.bn1)
                self.stem = ((F.conv_weight_2d(m.body.conv1.weight.detach().float())
                              * s_[None, :]).contiguous(), t_.detach().contiguous())
                self.layers = [[_MNv3Block(b) for b in getattr(m.body, f"layer{i}")]
                               for i in (1, 2, 3)]
                self.head = _Head(m, ("eca_40", "eca_80", "eca_160"), m.fpn.nlm)
            else:
                self.stem = F.pack_conv(m.body.conv1, m.body.bn1)
                self.layers = [[_R50Block(b) for b in getattr(m.body, f"layer{i}")]
                               for i in (1, 2, 3, 4)]
                self.head = _Head(m, ("eca_64", "eca_128", "eca_256"), m.fpn.Nlm)

    def forward(self, x):
        m = self.model
        if not isinstance(x, torch.Tensor) or not x.is_cuda or x.dtype != torch.float32:
            raise RuntimeError("RetinaFace.forward on the JABD HIP path needs a float32 GPU "
                               "tensor [B,3,H,W]; there is no CPU fallback")
        if x.dim() != 4 or x.shape[1] != 3:
            raise ValueError(f"expected input [B,3,H,W], got {tuple(x.shape)}")
        if m.training:
            from .train import train_forward
            return train_forward(m, self.kind, x)
        sig = _params_signature(m)
        if sig != self.sig:
            self._refresh()
            self.sig = _params_signature(m)
        x = x.contiguous()
        with torch.no_grad():
            if self.kind == "mnv3":
                s = F.stem(x, self.stem[0], self.stem[1], "hswish")
                feats = []
                for layer in self.layers:
                    for blk in layer:
                        s = blk.forward(s)
                    feats.append(s)
            else:
                s = F.conv(x, self.stem, stride=2, pad=3, act="relu", nchw_in=True)
                s = F.maxpool(s, 3, 2, 1)
                feats = []
                for li, layer in enumerate(self.layers):
                    for blk in layer:
                        s = blk.forward(s)
                    if li >= 1:
                        feats.append(s)
            return self.head.forward(feats, softmax=(m.mode != "train"))


def get_engine(model, kind):
    eng = model.__dict__.get("_engine")
    if eng is None or eng.kind != kind:
        eng = Engine(model, kind)
        model.__dict__["_engine"] = eng
    return eng
