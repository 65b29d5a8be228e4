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
  MobileNetV3-BECA (train_mobilenetV3_ecagai.py:319-435): the MobileNetV3
    plan with BECA gates (std pool + Hardsigmoid) on the head, bicubic
    up-sampling and the ch=40 NLM in the FPN.

There is no CPU path: inputs must be float32 tensors on the GPU.
"""
import os

import torch

from . import functional as F

NLM_SIZES_DEFAULT = (1, 4, 8, 12)
# MNv3 blocks run expand 1x1 + depthwise as one kernel (csrc/expdw.hip);
# JABD_FUSE_EXPAND_DW=0 selects the two-kernel path (A/B measurement, tests).
FUSE_EXPAND_DW = os.environ.get("JABD_FUSE_EXPAND_DW", "1") != "0"
# ... and the stride-2 blocks' dw3x3 skip branch into that kernel (it stages
# the same input tile); JABD_FUSE_SKIP=0 runs it as its own dw launch.
FUSE_SKIP = os.environ.get("JABD_FUSE_SKIP", "1") != "0"
# ... and a 16 -> 16 identity-residual block's project into the next block's
# fused kernel when that is the 3x3/s2 Cin-16 skip form (JABD-MNv3 blocks 1 -> 2:
# the 512^2 x 16 block output stays on chip); JABD_FUSE_PRE=0: separate launches
FUSE_PRE = os.environ.get("JABD_FUSE_PRE", "1") != "0"
# JABD_EVAL_STREAMS=2: eval batches of EVAL_SPLIT_MIN+ images run as image
# groups on their own HIP streams (Engine.run).  Off by default: at bs32
# 1024^2 two streams are +1.7% with weights_init's near-zero activations but
# -15% with O(1) activations (4540 -> 3840 img/s, same box): the overlapped
# launches cost more clock than the filled CUs gain once the data is real.
EVAL_STREAMS = int(os.environ.get("JABD_EVAL_STREAMS", "1"))
EVAL_SPLIT_MIN = int(os.environ.get("JABD_EVAL_SPLIT_MIN", "8"))
# Engine.run: activation elements one chunk of a batch may reach (32-bit offsets)
CHUNK_ELEMS = (1 << 31) - 1
# The head's three per-level ECA gates as one pool + gate launch pair
# (F.eca_gates_multi); JABD_GATES_MULTI=0 launches them level by level (A/B).
GATES_MULTI = os.environ.get("JABD_GATES_MULTI", "1") != "0"
# Heads of >= 128-channel levels (R50) as one GEMM + scatter instead of
# heads_kernel; JABD_HEADS_GEMM=0 for A/B.
HEADS_GEMM = os.environ.get("JABD_HEADS_GEMM", "1") != "0"
# JABD_SSH_TAIL=0: the 40-channel SSH's tail convs and the heads as separate
# launches (A/B against the fused ssh.hip kernel)
SSH_TAIL = os.environ.get("JABD_SSH_TAIL", "1") != "0"


def _w1d(eca):
    return eca.conv.weight.detach().reshape(-1).float().contiguous()


class SSHPack:
    """Eval packs of one SSH (nets/layers.py:37-68): the two branches that read
    the input (conv3X3, conv5X5_1) and the two that read t (conv5X5_2,
    conv7X7_2) run as one GEMM each with a split output (fused along N);
    every part's output channels are padded to a multiple of 4 for the vector
    epilogue (10-channel branches are stored as 12)."""

    def __init__(self, s):
        self.leaky = s.leaky
        q = s.conv5X5_1[0].out_channels
        self.q = q
        self.C = 2 * s.conv3X3[0].out_channels
        qp = (q + 3) // 4 * 4 if q % 4 else None
        q4 = (q + 3) // 4 * 4
        h2 = s.conv3X3[0].out_channels
        # (R50's 256-channel SSH keeps five GEMMs: each takes the 32x32 k x k
        # kernel, which the split output does not)
        self.split = h2 % 4 == 0 and s.conv3X3[0].in_channels % 32 != 0
        if self.split:
            self.packs = (
                F.pack_conv_cat([(s.conv3X3[0], s.conv3X3[1], None),
                                 (s.conv5X5_1[0], s.conv5X5_1[1], qp)]),
                F.pack_conv_cat([(s.conv5X5_2[0], s.conv5X5_2[1], q4),
                                 (s.conv7X7_2[0], s.conv7X7_2[1], qp)], cin_pad=qp),
                F.pack_conv(s.conv7x7_3[0], s.conv7x7_3[1], cin_pad=qp))
        else:
            self.packs = (F.pack_conv(s.conv3X3[0], s.conv3X3[1]),
                          F.pack_conv(s.conv5X5_1[0], s.conv5X5_1[1], cout_pad=qp),
                          F.pack_conv(s.conv5X5_2[0], s.conv5X5_2[1], cin_pad=qp),
                          F.pack_conv(s.conv7X7_2[0], s.conv7X7_2[1], cin_pad=qp, cout_pad=qp),
                          F.pack_conv(s.conv7x7_3[0], s.conv7x7_3[1], cin_pad=qp))

    def first(self, o, sc=None):
        """The split form's first GEMM alone: (relu(conv3X3) [B,h,w,C/2],
        t = leaky(conv5X5_1) [B,h,w,qp]) for the fused tail (ssh.hip)."""
        B, h, w, _ = o.shape
        ca = self.packs[0]
        c33 = torch.empty((B, h, w, self.C // 2), dtype=torch.float32, device=o.device)
        t = torch.empty((B, h, w, self.packs[1].Cin), dtype=torch.float32, device=o.device)
        F.conv(o, ca, pad=1, act="relu", ascale=sc, out=c33, out_c0=0, y2=t,
               nsplit=self.C // 2, act2="leaky", slope2=self.leaky)
        return c33, t

    def forward(self, o, sc=None):
        """o NHWC [B,h,w,Cin] (ECA gate `sc` [B,Cin] applied on load) -> relu(cat) NHWC."""
        B, h, w, _ = o.shape
        C = self.C
        dev = o.device
        feat = torch.empty((B, h, w, C), dtype=torch.float32, device=dev)
        if self.split:
            # feat = [conv3X3 (C/2) | conv5X5_2 (C/4) | conv7x7_3 (C/4)]; the
            # fused middle GEMM writes conv5X5_2 padded to a multiple of 4,
            # whose zero pad channels conv7x7_3 overwrites right after
            ca, cb, c73 = self.packs
            qp_ = cb.Cin
            t = torch.empty((B, h, w, qp_), dtype=torch.float32, device=dev)
            t2 = torch.empty((B, h, w, qp_), dtype=torch.float32, device=dev)
            F.conv(o, ca, pad=1, act="relu", ascale=sc, out=feat, out_c0=0, y2=t,
                   nsplit=C // 2, act2="leaky", slope2=self.leaky)
            F.conv(t, cb, pad=1, act="relu", out=feat, out_c0=C // 2, y2=t2,
                   nsplit=cb.Cout - qp_, act2="leaky", slope2=self.leaky)
            F.conv(t2, c73, pad=1, act="relu", out=feat, out_c0=3 * C // 4)
        else:
            c3, c51, c52, c72, c73 = self.packs
            F.conv(o, c3, pad=1, act="relu", ascale=sc, out=feat, out_c0=0)
            t = F.conv(o, c51, pad=1, act="leaky", slope=self.leaky, ascale=sc)
            F.conv(t, c52, pad=1, act="relu", out=feat, out_c0=C // 2)
            t2 = F.conv(t, c72, pad=1, act="leaky", slope=self.leaky)
            F.conv(t2, c73, pad=1, act="relu", out=feat, out_c0=3 * C // 4)
        return feat


class NlmPack:
    """Eval form of an NLM of any width (nets/retinaface_r.py:107-152;
    train_mobilenetV3_ecagai.py:182-234 for ch=40).  ch=4: the fused
    pool / apply kernels (head.hip).  Other widths: f_query as a 1x1 GEMM,
    PSP pooling of x then f_key / f_value on the S pooled rows (pooling is
    linear with unit-sum bins), the attention core (nlm_attn.hip), then W as a
    1x1 GEMM with the residual x added in its epilogue."""

    def __init__(self, nlm):
        self.ch = nlm.ch
        self.sizes = tuple(nlm.psp.sizes)
        if self.ch == 4:
            self.w = nlm_weights(nlm)
        else:
            self.q, self.k, self.v, self.W = (F.pack_conv(c) for c in
                                              (nlm.f_query, nlm.f_key, nlm.f_value, nlm.W))

    def forward(self, x, lateral=None):
        """NLM(x) (+ lateral), NHWC."""
        if self.ch == 4:
            y = F.nlm_fused(x, None, self.w, self.sizes)
            return F.add3(y, lateral, out=y) if lateral is not None else y
        B, h, w, C = x.shape
        S = sum(s * s for s in self.sizes)
        q = F.conv(x, self.q)
        pooled = F.adaptive_pool(x, self.sizes).view(B, S, 1, C)
        kp = F.conv(pooled, self.k).view(B, S, self.ch)
        vp = F.conv(pooled, self.v).view(B, S, self.ch)
        y = F.conv(F.nlm_attn(q, kp, vp), self.W, res=x)
        return F.add3(y, lateral, out=y) if lateral is not None else y


class FPNPack:
    """Eval packs of an FPN (nets/retinaface_r.py:154-207 with NLM `nlm`,
    nets/layers.py:70-119 with nlm=None, train_mobilenetV3_ecagai.py:237-285
    with bicubic up-sampling): 1x1 laterals (+BN+leaky), up-sample (+NLM) +
    add, 3x3 merges."""

    def __init__(self, fpn, nlm):
        self.leaky = fpn.leaky
        self.mode = getattr(fpn, "upsample_mode", "nearest")
        self.lat = [F.pack_conv(o[0], o[1]) for o in (fpn.output1, fpn.output2, fpn.output3)]
        self.merge1 = F.pack_conv(fpn.merge1[0], fpn.merge1[1])
        self.merge2 = F.pack_conv(fpn.merge2[0], fpn.merge2[1])
        self.nlm = NlmPack(nlm) if nlm is not None else None

    def _up(self, src, lateral):
        _, h, w, _ = lateral.shape
        if self.nlm is not None:
            if self.mode == "nearest" and self.nlm.ch == 4:  # one fused kernel pair
                return F.nlm_fused(src, lateral, self.nlm.w, self.nlm.sizes)
            return self.nlm.forward(F.upsample(src, h, w, self.mode), lateral)
        if self.mode == "nearest":
            return F.upsample_add(src, lateral)
        up = F.upsample(src, h, w, self.mode)
        return F.add3(up, lateral, out=up)

    def forward(self, feats, scales=(None, None, None)):
        o1, o2, o3 = [F.conv(f, pk, act="leaky", slope=self.leaky, ascale=sc)
                      for f, pk, sc in zip(feats, self.lat, scales)]
        o2 = F.conv(self._up(o3, o2), self.merge2, pad=1, act="leaky", slope=self.leaky)
        o1 = F.conv(self._up(o2, o1), self.merge1, pad=1, act="leaky", slope=self.leaky)
        return [o1, o2, o3]


def nlm_weights(nlm):
    C, ch = nlm.in_channels, nlm.ch
    d = lambda t: t.detach().float().contiguous()  # noqa: E731
    return (d(nlm.f_query.weight.view(ch, C)), d(nlm.f_query.bias),
            d(nlm.f_key.weight.view(ch, C)), d(nlm.f_key.bias),
            d(nlm.f_value.weight.view(ch, C)), d(nlm.f_value.bias),
            d(nlm.W.weight.view(C, ch)), d(nlm.W.bias))


def ssh_tail_pack(s, heads):
    """Packed weights of jabd_ssh_tail_heads_f32 for one level (csrc/ssh.hip):
    MFMA A fragments (lane = 16 g + j, float4 component e) of conv5X5_2,
    conv7X7_2, conv7x7_3 (BN folded) per tap — W[n = j][ch = 4g + e] — their
    biases per lane group, the heads' fragments over the k chunks (conv3X3
    0-15, conv3X3 16-19, conv5X5_2, conv7x7_3) x 2 output tiles, and the head
    biases.  None unless the SSH is the 40-channel one (branches 20/10/10)."""
    if (s.conv3X3[0].in_channels != 40 or s.conv3X3[0].out_channels != 20 or
            s.conv5X5_1[0].out_channels != 10 or tuple(heads[0].shape) != (32, 40)):
        return None
    dev = heads[0].device
    j = torch.arange(16, device=dev).view(1, 16, 1)        # [g, j, e]
    g = torch.arange(4, device=dev).view(4, 1, 1)
    e = torch.arange(4, device=dev).view(1, 1, 4)
    k = 4 * g + e                                          # channel of (g, e)
    convs, cbias = [], []
    for seq in (s.conv5X5_2, s.conv7X7_2, s.conv7x7_3):
        sc, sh = F.bn_fold(seq[1])
        w = (seq[0].weight.detach().float() * sc[:, None, None, None]).reshape(10, 10, 9)
        ok = (j < 10) & (k < 10)
        for p in range(9):
            frag = torch.where(ok, w[j.clamp(max=9), k.clamp(max=9), p], torch.zeros((), device=dev))
            convs.append(frag.reshape(64, 4))              # lane = 16 g + j
        b16 = torch.zeros(16, device=dev)
        b16[:10] = sh.detach().float()
        cbias.append(b16.view(4, 4))
    wh, bh = heads
    hfr = []
    for kc in range(4):
        if kc == 0:
            ch, ok = k, k < 16
        elif kc == 1:
            ch, ok = 16 + k, k < 4
        else:
            ch, ok = (20 if kc == 2 else 30) + k, k < 10
        for nt in range(2):
            frag = torch.where(ok & (j >= 0), wh[16 * nt + j, ch.clamp(max=39)],
                               torch.zeros((), device=dev))
            hfr.append(frag.reshape(64, 4))
    wb = torch.cat([torch.cat(convs).reshape(-1), torch.cat(cbias).reshape(-1),
                    torch.cat(hfr).reshape(-1), bh.reshape(2, 4, 4).reshape(-1)]).contiguous()
    if wb.numel() != int(F.lib().jabd_ssh_tail_weight_floats()):
        raise RuntimeError("ssh_tail_pack: layout mismatch with libjabd")
    return wb


def heads_pack(m, i):
    convs = (m.BboxHead[i].conv1x1, m.ClassHead[i].conv1x1, m.LandmarkHead[i].conv1x1)
    w = torch.cat([c.weight.detach().float().reshape(c.weight.shape[0], -1) for c in convs])
    b = torch.cat([c.bias.detach().float() for c in convs])
    return w.contiguous(), b.contiguous()


class _Head:
    """ECA -> FPN(+NLM) -> ECA -> SSH -> heads, shared by both detectors.
    The FPN and SSH packs are the modules' own cached packs (also used when
    those modules run standalone)."""

    def __init__(self, m, eca_names, nlm_name, dev, gate="sigmoid"):
        self.gate = gate  # "sigmoid": mean-pool ECA; "beca": std-pool + Hardsigmoid
        self.eca_in = [_w1d(getattr(m, n)) for n in eca_names]
        self.fpn = m.fpn._jabd_cached(dev, lambda: FPNPack(m.fpn, getattr(m.fpn, nlm_name)))
        self.eca_fpn = _w1d(m.eca_fpn)
        self.ssh = [s._jabd_cached(dev, lambda s=s: SSHPack(s)) for s in (m.ssh1, m.ssh2, m.ssh3)]
        self.heads = [heads_pack(m, i) for i in range(3)]
        # the 40-channel SSH's tail + heads as one launch per level (ssh.hip)
        self.tails = [ssh_tail_pack(s, self.heads[i]) if SSH_TAIL and p.split else None
                      for i, (s, p) in enumerate(zip((m.ssh1, m.ssh2, m.ssh3), self.ssh))]
        # wide levels (R50: 256 channels): the three heads as one MFMA GEMM
        # plus a scatter; heads_kernel's per-position channel loop is serial
        self.heads_gemm = [
            F.pack_conv_cat([(m.BboxHead[i].conv1x1, None, None), (m.ClassHead[i].conv1x1, None, None),
                             (m.LandmarkHead[i].conv1x1, None, None)])
            if HEADS_GEMM and m.BboxHead[i].conv1x1.in_channels >= 128 else None
            for i in range(3)]

    def _gate(self, f, w1d):
        if self.gate == "beca":
            from . import modules as M
            return M.beca_gate(f, w1d)
        return F.eca_gate(F.channel_sums(f), f.shape[1] * f.shape[2], w1d, "sigmoid")

    def _gates(self, fs, w1ds):
        """The gates of the three levels; mean-pool ECA as one multi-tensor
        pool + gate pair of launches (F.eca_gates_multi)."""
        if GATES_MULTI and self.gate == "sigmoid" and all(f.stride(3) == 1 for f in fs):
            sc = F.eca_gates_multi(list(fs), list(w1ds), "sigmoid")
            if sc is not None:
                return sc
        return [self._gate(f, w1d) for f, w1d in zip(fs, w1ds)]

    def forward(self, feats, softmax, out=None):
        B = feats[0].shape[0]
        scales = self._gates(feats, self.eca_in)
        levels = self.fpn.forward(feats, scales)
        A = sum(2 * o.shape[1] * o.shape[2] for o in levels)
        dev = levels[0].device
        if out is not None:  # batch slices of the caller's outputs
            loc, conf, landm = out
            if loc.shape[1] != A:
                raise RuntimeError(f"engine: anchor count {loc.shape[1]} != {A} of the levels")
        else:
            loc = torch.empty((B, A, 4), dtype=torch.float32, device=dev)
            conf = torch.empty((B, A, 2), dtype=torch.float32, device=dev)
            landm = torch.empty((B, A, 10), dtype=torch.float32, device=dev)
        a_off = 0
        scs = self._gates(levels, [self.eca_fpn] * len(levels))
        for i, o in enumerate(levels):
            _, h, w, C = o.shape
            if self.tails[i] is not None:
                c33, t = self.ssh[i].first(o, scs[i])
                F.ssh_tail_heads(c33, t, self.tails[i], self.ssh[i].leaky, loc, conf, landm,
                                 a_off, softmax)
                a_off += 2 * h * w
                continue
            feat = self.ssh[i].forward(o, scs[i])
            if self.heads_gemm[i] is not None:
                F.heads_scatter(F.conv(feat, self.heads_gemm[i]), loc, conf, landm, a_off, softmax)
            else:
                wt, bs = self.heads[i]
                F.heads(feat, wt, bs, loc, conf, landm, a_off, softmax)
            a_off += 2 * h * w
        return loc, conf, landm


class _MNv3Block:
    """Eval plan of one MobileNetV3 inverted-residual block (nets/mobilenetV3.py:
    Block_eca :94-150, Block :35-91, Block_eca_G :152-208): fused expand 1x1 +
    depthwise kxk (+ECA pool partials), the channel gate (ECA / SE / BECA) as a
    [B, E] scale the project GEMM applies on its operand load, the skip branch
    K-concatenated or added in the project GEMM's epilogue."""

    def __init__(self, blk):
        self.k, self.stride, self.act = blk.kernel_size, blk.stride, blk.act_name
        self.expand = F.pack_conv(blk.conv1, blk.bn1)
        self.dw_w, self.dw_b = F.pack_dw(blk.conv2, blk.bn2)
        self.gate = getattr(blk, "gate_kind", "eca")
        self.blk = blk
        if self.gate in ("eca", "beca"):
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

    def _scale(self, d, part):
        if self.gate == "eca":
            return F.eca_gate(part, d.shape[1] * d.shape[2], self.eca, "hsigmoid")
        from . import modules as M
        if self.gate == "se":
            return M.se_scale_eval(self.blk.se, d, self.blk)
        if self.gate == "beca":
            return M.beca_gate(d, self.eca)
        return None

    def can_defer(self):
        """This block's project can run inside the next block's fused kernel:
        ECA gate, identity residual, a 16 -> 16 1x1 with a folded bias."""
        pk = self.project
        return (FUSE_PRE and FUSE_EXPAND_DW and self.gate == "eca" and self.kind == "identity" and
                pk.KH == 1 and pk.KW == 1 and pk.Cin == 16 and pk.Cout == 16 and not pk.Cin2 and
                pk.bias is not None)

    def takes_pre(self):
        """The fused kernel can take the previous block's project: the 3x3/s2
        skip form over 16 input channels, and nothing after it reads this
        block's input (its skip branch runs inside that kernel)."""
        return (FUSE_EXPAND_DW and FUSE_SKIP and self.stride == 2 and self.k == 3 and
                self.skip_dw is not None and self.kind in ("dw_concat", "dw_residual") and
                self.expand.Cin == 16 and self.expand.KH == 1 and not self.expand.Cin2)

    def front(self, x):
        """Expand + depthwise + ECA gate of this block; its project is handed
        to the next block's kernel: (d, (project, gate, residual, act))."""
        d, part = F.expand_dw(x, self.expand, self.dw_w, self.dw_b, self.k, self.stride,
                              act=self.act, partials=True)
        return d, (self.project, self._scale(d, part), x, self.act)

    def forward(self, x, pre=None):
        t = None
        if pre is not None:  # x: the previous block's (d, project) from front()
            d_prev, pspec = x, pre
            r = F.expand_dw(d_prev, self.expand, self.dw_w, self.dw_b, self.k, self.stride,
                            act=self.act, partials=self.gate == "eca", skip=self.skip_dw,
                            pre=pspec)
            d, part, t = r
        elif FUSE_EXPAND_DW:
            fuse_skip = FUSE_SKIP and self.skip_dw is not None and self.stride == 2
            r = F.expand_dw(x, self.expand, self.dw_w, self.dw_b, self.k, self.stride,
                            act=self.act, partials=self.gate == "eca",
                            skip=self.skip_dw if fuse_skip else None)
            d, part = r[0], r[1]
            if fuse_skip:
                t = r[2]
        else:
            e = F.conv(x, self.expand, act=self.act)
            d, part = F.dwconv(e, self.dw_w, self.dw_b, self.k, self.stride, act=self.act,
                               partials=self.gate == "eca")
        sc = self._scale(d, part)
        if self.kind == "identity":
            return F.conv(d, self.project, act=self.act, ascale=sc, res=x)
        if self.kind == "concat":
            return F.conv(d, self.project, act=self.act, ascale=sc, x2=x)
        if t is None:
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


def mnv3_stages(body):
    """The three block lists of a MobileNetV3 detector body (layer1..3 of
    MobileNetV3_Large_eca, or MobileNetV3_Small's tapped bneck)."""
    if hasattr(body, "stages"):
        return body.stages()
    return [list(getattr(body, f"layer{i}")) for i in (1, 2, 3)]


class Engine:
    """The eval-mode plan of one RetinaFace on one device (packs built once per
    generation, see hipmodule.py)."""

    def __init__(self, model, kind, dev):
        m = model
        self.kind = kind
        if kind == "mnv3":
            s_, t_ = F.bn_fold(m.body.bn1)
            self.stem = ((F.conv_weight_2d(m.body.conv1.weight.detach().float())
                          * s_[None, :]).contiguous(), t_.detach().contiguous())
            self.layers = [[b._jabd_cached(dev, lambda b=b: _MNv3Block(b)) for b in stage]
                           for stage in mnv3_stages(m.body)]
            self.head = _Head(m, getattr(m, "eca_names", ("eca_40", "eca_80", "eca_160")), "nlm",
                              dev, gate=getattr(m, "head_gate", "sigmoid"))
            # the split is offered for the JABD-MNv3 detector (ECA blocks,
            # mean-pool ECA head) only; MobileNetV3_Small (SE gates, 4 ms/step
            # of small launches) loses 28% with it and the BECA head is neutral
            self.split_ok = (self.head.gate == "sigmoid" and
                             all(b.gate == "eca" for layer in self.layers for b in layer))
        else:
            self.stem = F.pack_conv(m.body.conv1, m.body.bn1)
            self.layers = [[b._jabd_cached(dev, lambda b=b: _R50Block(b))
                            for b in getattr(m.body, f"layer{i}")] for i in (1, 2, 3, 4)]
            self.head = _Head(m, ("eca_64", "eca_128", "eca_256"), "Nlm", dev)
            self.split_ok = False  # compute-bound convs; not measured split

    def run(self, x, softmax):
        """Forward of a batch.  From EVAL_SPLIT_MIN images up, the batch is
        split into EVAL_STREAMS image groups, each run on its own HIP stream
        (every op is per image, so the groups are independent): the small
        launches of one group (ECA gates, pools, the 32x32 / 64x64 head convs,
        NLM, heads) run beside the large convs of the other instead of leaving
        most of the CUs idle.  The heads write straight into batch slices of
        one set of outputs."""
        B = x.shape[0]
        # the kernels index a batch's activations with 32-bit element offsets
        # (and expand_dw reads its input through a < 4 GiB buffer descriptor):
        # the largest stored activation is <= 16*H*W elements per image (R50
        # layer1: 256 channels at H/4 x W/4), so larger batches run in chunks
        per_img = 16 * x.shape[2] * x.shape[3]
        chunk = max(1, CHUNK_ELEMS // per_img)
        if B > chunk:
            A = self.anchors(x.shape[2], x.shape[3])
            out = tuple(torch.empty((B, A, k), dtype=torch.float32, device=x.device)
                        for k in (4, 2, 10))
            for b0 in range(0, B, chunk):
                b1 = min(B, b0 + chunk)
                self._run(x[b0:b1], softmax, out=tuple(o[b0:b1] for o in out))
            return out
        n = min(EVAL_STREAMS, B) if B >= EVAL_SPLIT_MIN and self.split_ok else 1
        if n <= 1:
            return self._run(x, softmax)
        cur = torch.cuda.current_stream(x.device)
        if getattr(self, "_streams", None) is None or len(self._streams) < n:
            self._streams = [torch.cuda.Stream(device=x.device) for _ in range(n)]
        bounds = [B * i // n for i in range(n + 1)]
        with torch.no_grad():
            H, W = x.shape[2], x.shape[3]
            A = self.anchors(H, W)
            dev = x.device
            out = (torch.empty((B, A, 4), dtype=torch.float32, device=dev),
                   torch.empty((B, A, 2), dtype=torch.float32, device=dev),
                   torch.empty((B, A, 10), dtype=torch.float32, device=dev))
            for i in range(n):
                st = self._streams[i]
                st.wait_stream(cur)
                b0, b1 = bounds[i], bounds[i + 1]
                with torch.cuda.stream(st):
                    self._run(x[b0:b1], softmax, out=tuple(o[b0:b1] for o in out))
            for i in range(n):
                cur.wait_stream(self._streams[i])
        return out

    def anchors(self, H, W):
        """Anchor count of an H x W input: 2 per cell of the stride-8/16/32 maps
        (the detector's own conv arithmetic, pad 1, kernel 3, stride 2)."""
        def down(v, times):
            for _ in range(times):
                v = (v + 2 - 3) // 2 + 1
            return v
        if self.kind == "mnv3":
            sizes = [(down(H, t), down(W, t)) for t in (3, 4, 5)]
        else:  # R50: 7x7/s2 stem, 3x3/s2 max-pool, then /2 per stage
            h, w = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
            h, w = down(h, 1), down(w, 1)
            sizes = [(down(h, t), down(w, t)) for t in (1, 2, 3)]
        return sum(2 * a * b for a, b in sizes)

    def _run(self, x, softmax, out=None):
        with torch.no_grad():
            if self.kind == "mnv3":
                s = F.stem(x, self.stem[0], self.stem[1], "hswish")
                feats = []
                for layer in self.layers:
                    pre = None
                    for i, blk in enumerate(layer):
                        nxt = layer[i + 1] if i + 1 < len(layer) else None
                        if pre is None and nxt is not None and blk.can_defer() and \
                                nxt.takes_pre():
                            s, pre = blk.front(s)   # s: this block's d, for the next kernel
                            continue
                        s = blk.forward(s, pre=pre)
                        pre = None
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
            return self.head.forward(feats, softmax=softmax, out=out)


def _check_input(x):
    if not isinstance(x, torch.Tensor) or not x.is_cuda or x.dtype != torch.float32:
        raise RuntimeError("RetinaFace.forward on the JABD HIP path needs a float32 GPU "
                           "tensor [B,3,H,W]; there is no CPU fallback")
    if x.dim() != 4 or x.shape[1] != 3:
        raise ValueError(f"expected input [B,3,H,W], got {tuple(x.shape)}")


def retinaface_forward(model, kind, x):
    """RetinaFace.forward: the fused eval plan, or the training graph.

    `model` is the module being called — under nn.DataParallel that is the
    replica on x's device, so training binds autograd to the replica's
    broadcast parameters and eval uses packs built from them (cached per
    device on the shared cache of the original)."""
    _check_input(x)
    if model.training:
        from .train import train_forward
        return train_forward(model, kind, x)
    eng = model._jabd_cached(x.device, lambda: Engine(model, kind, x.device), tag="engine")
    return eng.run(x.contiguous(), softmax=(model.mode != "train"))
