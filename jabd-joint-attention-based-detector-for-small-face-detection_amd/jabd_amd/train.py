"""Training-mode forward/backward of the JABD detectors on the HIP path (A11).

`train_forward(model, kind, x)` runs RetinaFace.forward in training mode
(BatchNorm2d with batch statistics and running-buffer updates, as
`loss.backward()` at train_mobilenetV3_ecagai.py:532 expects) as a graph of
torch.autograd.Functions whose forward AND backward passes are libjabd
kernels (fp32, NHWC):

  ConvFn      implicit-GEMM conv (MFMA); dgrad = transposed-conv GEMM,
              wgrad = MFMA weight-gradient kernel
  EcaConvFn   conv(x * ECA(x)) — the ECA gate applied on the GEMM's operand
              load; backward through the gate, Conv1d and average pool
  BnActFn     batch-stat BN + activation (+ the block's residual add)
  DwConvFn    depthwise conv; dgrad/wgrad kernels
  NlmFn       CSAF non-local block fused with the up-sample and lateral add
  NlmAttnFn   attention core of the other NLM widths (ch=40, BECA variant)
  UpsampleFn  nearest / bicubic(align_corners) up-sampling; Add3Fn adds
  SshTailFn   SSH's three BN branches written into one concatenated tensor
  HeadsFn     the three 1x1 heads of all levels -> (loc, conf, landm)
  MaxPoolFn   ResNet stem max pool

Torch is used only for allocation, views and a few tiny reductions of
kernel partials.  There is no CPU path.
"""
import ctypes
import threading
import weakref

import torch

from . import functional as F
from ._lib import ConvArgs, call, lib

ACT = F.ACT
# MobileNetV3 Block_eca training as one autograd node (MNv3BlockFn);
# JABD_FUSED_BLOCKS=0 selects the per-op graph (A/B measurement, tests).
FUSED_BLOCKS = __import__("os").environ.get("JABD_FUSED_BLOCKS", "1") != "0"
# JABD_ECA_WGRAD=0: the ECA block backward takes sum(da * d) from its own pass (A/B)
ECA_WGRAD = __import__("os").environ.get("JABD_ECA_WGRAD", "1") != "0"
# JABD_ECA_SUMS=0: the ECA pool of a block reads d in its own pass (A/B)
ECA_SUMS = __import__("os").environ.get("JABD_ECA_SUMS", "1") != "0"
# JABD_DW_BN_FUSE=0: bn1's backward partials from their own pass over de and
# e_pre instead of the depthwise data-gradient kernel, and bn2's statistics
# from their own pass over d_pre instead of the depthwise forward, and bn1's
# statistics from their own pass over e_pre instead of conv1's streaming kernel
# (A/B)
DW_BN_FUSE = __import__("os").environ.get("JABD_DW_BN_FUSE", "1") != "0"
# R50 bn1 / bn2 backward sums in the data-gradient GEMM's epilogue
# (_dgrad_bn_sums); JABD_BN_BWD_EPI=0 keeps the separate reduction pass (A/B)
BN_BWD_EPI = __import__("os").environ.get("JABD_BN_BWD_EPI", "1") != "0"
# JABD_DW_BNIN=0: bn1 + act written out as e and read by conv2 and its weight
# gradient, instead of applied on their loads from e_pre (A/B; needs
# DW_BN_FUSE).  Only the 3x3 stride-2 blocks take it: their kernels load each
# input element ~1.7 times, so the on-load BN stays under the HBM time it
# saves; 3x3/s1 (4.5 loads per element) and 5x5 (3.4-10) turn VALU-bound
# and lose (r03 C4 profile).
DW_BNIN = __import__("os").environ.get("JABD_DW_BNIN", "1") != "0"
# JABD_DW_BNIN_S1=1: the 3x3 stride-1 blocks take bn1 + act on load as well
# (their forward and weight-gradient kernels are row walkers now, ~1.6 loads
# per input element).  Measured neutral (C4 52.8 vs 52.9 ms/step: the saved
# apply pass is spent in the walkers' VALU), so off by default; it does save
# the stored e of those blocks.
DW_BNIN_S1 = __import__("os").environ.get("JABD_DW_BNIN_S1", "0") == "1"
# JABD_DGBN_RECOMPUTE=0: bn1's backward stores de and applies from it instead
# of recomputing de in a second depthwise pass (A/B)
DGBN_RECOMPUTE = __import__("os").environ.get("JABD_DGBN_RECOMPUTE", "1") != "0"


_ZEROS = {}


def _zeros(n, dev):
    """A read-only zero vector of >= n floats per device (allocated once)."""
    key = str(dev)
    t = _ZEROS.get(key)
    if t is None or t.numel() < n:
        t = torch.zeros(max(n, 64), dtype=torch.float32, device=dev)
        _ZEROS[key] = t
    return t


def _st():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t):
    return t.data_ptr() if t is not None else None


# ----------------------------------------------------------------------------- packing cache
_PACK = {}  # id(Parameter) -> (weakref to it, {(version, ptr, transposed): PackedConv})


def _packed(weight, transposed):
    """PackedConv of a raw (unfolded) conv weight; transposed = data-gradient form.

    Cached per live Parameter object (weak key, so a freed parameter's address
    can never hit a stale entry) and per version (an optimizer step bumps it);
    derived tensors are packed per call."""
    cache = None
    key = (weight._version, weight.data_ptr(), transposed)
    if isinstance(weight, torch.nn.Parameter):
        ent = _PACK.get(id(weight))
        if ent is None or ent[0]() is not weight:  # new or recycled id: start fresh
            ent = (weakref.ref(weight, lambda _r, i=id(weight): _PACK.pop(i, None)), {})
            _PACK[id(weight)] = ent
        cache = ent[1]
        pk = cache.get(key)
        if pk is not None:
            return pk
    # transposed: [Cin][Cout][KH][KW] is the dgrad GEMM's "weight"
    pk = F.pack_weight_device(weight, transposed)
    if cache is not None:
        if len(cache) > 4:  # stale versions
            cache.clear()
        cache[key] = pk
    return pk


_REPACK_TABLES = {}  # job-table key -> [(device jobs, device starts, njobs, total)] per launch
REPACK_MAX_JOBS = 1024  # kPackMaxJobs in csrc/conv32.hip


def repack(params):
    """After an optimizer step changed `params` in place (and bumped their
    versions): rewrite every cached training pack of them in its existing
    buffers with ONE launch (jabd_conv_pack_multi_f32) and re-key the cache to
    the new versions, instead of one jabd_conv_pack_f32 launch per weight and
    form at the next forward.  Keeps the newest pack per form; a parameter
    with no cached pack is packed lazily by _packed as before.  (A graph
    retained across the step would see the new weights in its packs, as
    autograd sees in-place parameter updates.)"""
    rows, fixups = [], []
    for w in params:
        ent = _PACK.get(id(w))
        if ent is None or ent[0]() is not w or not ent[1]:
            continue
        cache = ent[1]
        newest = {}
        for key, pk in cache.items():
            ver, ptr, tr = key
            if ptr == w.data_ptr() and (tr not in newest or ver > newest[tr][0]):
                newest[tr] = (ver, pk)
        if not newest or not w.is_contiguous() or w.dtype != torch.float32:
            continue
        cout, cin, kh, kw = w.shape
        for tr, (_, pk) in newest.items():
            k8 = pk.w32.shape[0] if pk.w32 is not None else 0
            nt32 = pk.w32.shape[1] if pk.w32 is not None else 0
            rows.append((w.data_ptr(), pk.w.data_ptr(), _p(pk.w32) or 0, cout, cin, kh * kw,
                         1 if tr else 0, pk.Kc, pk.Ntiles, k8, nt32))
        fixups.append((w, cache, newest))
    if not rows:
        return 0
    key = tuple(rows)
    tabs = _REPACK_TABLES.get(key)
    if tabs is None:
        # the kernel takes at most REPACK_MAX_JOBS jobs per launch (its job
        # starts live in LDS): larger models launch once per chunk of rows
        dev = fixups[0][0].device
        tabs = []
        for c0 in range(0, len(rows), REPACK_MAX_JOBS):
            chunk = rows[c0:c0 + REPACK_MAX_JOBS]
            starts = [0]
            for r in chunk:
                starts.append(starts[-1] + (r[7] * r[8] + r[9] * r[10]) * 64)
            tabs.append((torch.tensor(chunk, dtype=torch.int64).to(dev),
                         torch.tensor(starts, dtype=torch.int64).to(dev), len(chunk), starts[-1]))
        if len(_REPACK_TABLES) > 8:
            _REPACK_TABLES.clear()
        _REPACK_TABLES[key] = tabs
    for jobs, starts, n, total in tabs:
        call("jabd_conv_pack_multi_f32", jobs.data_ptr(), starts.data_ptr(), n, total, _st())
    for w, cache, newest in fixups:
        cache.clear()
        for tr, (_, pk) in newest.items():
            cache[(w._version, w.data_ptr(), tr)] = pk
    return len(rows)


def _conv_args(x, pk, y, stride, pad, nchw_in=False, ascale=None, tconv=False, OH=None, OW=None):
    a = ConvArgs()
    if nchw_in:
        B, cin, H, W = x.shape
        a.x, a.x_bs, a.x_ps = x.data_ptr(), cin * H * W, 1
    else:
        B, H, W, ctot = x.shape
        a.x, a.x_bs, a.x_ps = x.data_ptr(), H * W * ctot, ctot
    a.B, a.H, a.W, a.Cin = B, H, W, pk.Cin
    if ascale is not None:
        a.ascale, a.ascale_bs = ascale.data_ptr(), ascale.shape[1]
    a.w = pk.w.data_ptr()
    a.y, a.y_bs, a.y_ps, a.y_c0 = y.data_ptr(), y.stride(0), y.shape[3], 0
    a.OH = y.shape[1] if OH is None else OH
    a.OW = y.shape[2] if OW is None else OW
    a.Cout, a.Ntiles, a.tn, a.Kc = pk.Cout, pk.Ntiles, pk.tn, pk.Kc
    a.KH, a.KW, a.stride, a.pad = pk.KH, pk.KW, stride, pad
    a.nchw_in = 1 if nchw_in else 0
    a.tconv = 1 if tconv else 0
    if pk.w32 is not None and not nchw_in and (not tconv or stride <= 2):
        a.w32, a.ntiles32, a.tn32 = pk.w32.data_ptr(), pk.ntiles32, pk.tn32
    return a


def _wgrad(x, dy, weight, stride, pad, nchw_in=False, ascale=None):
    """dW (torch layout) of conv(x[*ascale]) given dY (NHWC)."""
    cout, cin, kh, kw = weight.shape
    a = ConvArgs()
    if nchw_in:
        B, _, H, W = x.shape
        a.x, a.x_bs, a.x_ps = x.data_ptr(), cin * H * W, 1
    else:
        B, H, W, ctot = x.shape
        a.x, a.x_bs, a.x_ps = x.data_ptr(), H * W * ctot, ctot
    a.B, a.H, a.W, a.Cin = B, H, W, cin
    if ascale is not None:
        a.ascale, a.ascale_bs = ascale.data_ptr(), ascale.shape[1]
    a.y, a.y_bs, a.y_ps, a.y_c0 = dy.data_ptr(), dy.stride(0), dy.shape[3], 0
    a.OH, a.OW, a.Cout = dy.shape[1], dy.shape[2], cout
    a.KH, a.KW, a.stride, a.pad = kh, kw, stride, pad
    a.nchw_in = 1 if nchw_in else 0
    nparts = int(lib().jabd_conv_wgrad_part_floats(ctypes.byref(a)))
    part = torch.empty(max(nparts, 1), dtype=torch.float32, device=dy.device)
    dw = torch.empty_like(weight, dtype=torch.float32)
    call("jabd_conv_wgrad_f32", ctypes.byref(a), part.data_ptr(), dw.data_ptr(), _st())
    return dw


def _chan_sum(t):
    """Per-channel sum of an NHWC tensor (bias gradients)."""
    return F.channel_total(t)


def _wgrad_eca(x, dy, weight, scale):
    """(dW, ds) of p = conv1x1(x * scale[b][c]) with ds[b][c] = sum_hw(da * x):
    jabd_conv_wgrad_eca_f32, or None when the shape does not qualify."""
    cout, cin = weight.shape[0], weight.shape[1]
    B, H, W, ctot = x.shape
    if ctot != cin or dy.shape[3] != cout:
        return None
    a = ConvArgs()
    a.x, a.x_bs, a.x_ps = x.data_ptr(), H * W * cin, cin
    a.B, a.H, a.W, a.Cin = B, H, W, cin
    a.y, a.y_bs, a.y_ps, a.y_c0 = dy.data_ptr(), dy.stride(0), cout, 0
    a.OH, a.OW, a.Cout = H, W, cout
    a.KH, a.KW, a.stride, a.pad = 1, 1, 1, 0
    nparts = int(lib().jabd_conv_wgrad_eca_part_floats(ctypes.byref(a)))
    if nparts <= 0:
        return None
    part = torch.empty(nparts, dtype=torch.float32, device=dy.device)
    dw = torch.empty_like(weight, dtype=torch.float32)
    ds = torch.empty((B, cin), dtype=torch.float32, device=dy.device)
    w = weight.detach().reshape(cout, cin).float().contiguous()
    call("jabd_conv_wgrad_eca_f32", ctypes.byref(a), scale.data_ptr(), w.data_ptr(),
         part.data_ptr(), dw.data_ptr(), ds.data_ptr(), _st())
    return dw, ds


def _dgrad(dy, weight, stride, pad, H, W):
    pk = _packed(weight, transposed=True)
    B = dy.shape[0]
    dx = torch.empty((B, H, W, pk.Cout), dtype=torch.float32, device=dy.device)
    # a 1x1 / stride-1 data gradient is a plain 1x1 conv with the transposed
    # weights (takes the conv1x1 fast path)
    plain = pk.KH == 1 and pk.KW == 1 and stride == 1 and pad == 0
    a = _conv_args(dy, pk, dx, stride, pad, tconv=not plain, OH=H, OW=W)
    call("jabd_conv2d_nhwc_f32", ctypes.byref(a), _st())
    return dx


# ----------------------------------------------------------------------------- functions
class ConvFn(torch.autograd.Function):
    """y = conv(x, weight) [+ bias]; x NHWC (or the NCHW network input)."""

    @staticmethod
    def forward(ctx, x, weight, bias, stride, pad, nchw_in):
        pk = _packed(weight, transposed=False)
        if nchw_in:
            B, _, H, W = x.shape
        else:
            B, H, W, _ = x.shape
        OH = (H + 2 * pad - pk.KH) // stride + 1
        OW = (W + 2 * pad - pk.KW) // stride + 1
        y = torch.empty((B, OH, OW, pk.Cout), dtype=torch.float32, device=x.device)
        if (nchw_in and pk.KH == 3 and stride == 2 and pad == 1 and pk.Cin == 3
                and pk.Cout == 16):
            wd = weight.detach()
            wt = torch.empty((27, 16), dtype=torch.float32, device=x.device)
            call("jabd_conv_w2d_f32", wd.data_ptr(), 16, 3, 9, wt.data_ptr(), _st())
            zb = _zeros(16, x.device)
            call("jabd_stem_nchw_f32", x.data_ptr(), B, H, W, wt.data_ptr(), zb.data_ptr(),
                 ACT["none"], y.data_ptr(), _st())
        else:
            a = _conv_args(x, pk, y, stride, pad, nchw_in=nchw_in)
            if bias is not None:
                b = bias.detach().float().contiguous()
                a.bias = b.data_ptr()
            call("jabd_conv2d_nhwc_f32", ctypes.byref(a), _st())
        ctx.save_for_backward(x, weight)
        ctx.cfg = (stride, pad, nchw_in, bias is not None, H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        stride, pad, nchw_in, has_bias, H, W = ctx.cfg
        dy = dy.contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            dx = _dgrad(dy, weight, stride, pad, H, W)
            if nchw_in:  # a network input that requires grad: hand it back as NCHW
                dx = dx.permute(0, 3, 1, 2).contiguous()
        dw = _wgrad(x, dy, weight, stride, pad, nchw_in) if ctx.needs_input_grad[1] else None
        db = _chan_sum(dy) if has_bias and ctx.needs_input_grad[2] else None
        return dx, dw, db, None, None, None


class EcaConvFn(torch.autograd.Function):
    """y = conv(x * eca(x), weight): ECA (mean pool -> Conv1d -> gate) of x,
    applied on the GEMM's operand load (nets/mobilenetV3.py:343-348 then the
    consumer conv; nets/retinaface_r.py:219-224 for the head ECAs)."""

    @staticmethod
    def forward(ctx, x, w1d, weight, stride, pad, gate):
        B, H, W, C = x.shape
        w1 = w1d.detach().reshape(-1).float().contiguous()
        scale, mean = F.eca_gate(F.channel_sums(x), H * W, w1, gate, return_mean=True)
        if gate == "hsigmoid":
            F.tap("eca", gate, mean, w1)
        pk = _packed(weight, transposed=False)
        OH = (H + 2 * pad - pk.KH) // stride + 1
        OW = (W + 2 * pad - pk.KW) // stride + 1
        y = torch.empty((B, OH, OW, pk.Cout), dtype=torch.float32, device=x.device)
        a = _conv_args(x, pk, y, stride, pad, ascale=scale)
        call("jabd_conv2d_nhwc_f32", ctypes.byref(a), _st())
        ctx.save_for_backward(x, w1d, weight, scale, mean)
        ctx.cfg = (stride, pad, gate, H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w1d, weight, scale, mean = ctx.saved_tensors
        stride, pad, gate, H, W = ctx.cfg
        dy = dy.contiguous()
        B, _, _, C = x.shape
        da = _dgrad(dy, weight, stride, pad, H, W)          # grad of x*scale
        dw = _wgrad(x, dy, weight, stride, pad, ascale=scale)
        w1 = w1d.detach().reshape(-1).float().contiguous()
        k = w1.numel()
        HW = H * W
        nblk = max(1, min(64, HW // 256))
        part = torch.empty((B, nblk, C), dtype=torch.float32, device=x.device)
        dmean = torch.empty((B, C), dtype=torch.float32, device=x.device)
        dw1_img = torch.empty((B, k), dtype=torch.float32, device=x.device)
        dx = torch.empty_like(x)
        dw1 = torch.empty(k, dtype=torch.float32, device=x.device)
        call("jabd_eca_bwd_f32", da.data_ptr(), x.data_ptr(), B, HW, C, scale.data_ptr(),
             mean.data_ptr(), w1.data_ptr(), k, ACT[gate], part.data_ptr(), nblk,
             dmean.data_ptr(), dw1_img.data_ptr(), dx.data_ptr(), dw1.data_ptr(), _st())
        return dx, dw1.view_as(w1d), dw, None, None, None


class BnActFn(torch.autograd.Function):
    """y = act(BN_train(x) [+ res]); updates the running buffers in place."""

    @staticmethod
    def forward(ctx, x, gamma, beta, res, rmean, rvar, act, slope, momentum, eps):
        B, H, W, C = x.shape
        M = B * H * W
        nblk = int(lib().jabd_bn_nblk(M, C))
        part = torch.empty((nblk, 2, C), dtype=torch.float32, device=x.device)
        mean = torch.empty(C, dtype=torch.float32, device=x.device)
        invstd = torch.empty_like(mean)
        call("jabd_bn_stats_f32", x.data_ptr(), C, M, C, part.data_ptr(), mean.data_ptr(),
             invstd.data_ptr(), _p(rmean), _p(rvar), float(momentum), float(eps), _st())
        F.tap("stats", "bn_stats", x, mean, invstd, eps)
        y = torch.empty_like(x)
        g = gamma.detach().contiguous()
        b = beta.detach().contiguous()
        call("jabd_bn_act_fwd_f32", x.data_ptr(), C, M, C, mean.data_ptr(), invstd.data_ptr(),
             g.data_ptr(), b.data_ptr(), _p(res), C, ACT[act], float(slope), y.data_ptr(), C, 0,
             _st())
        if act != "none":
            F.tap("bn", act, slope, x, mean, invstd, g, b, res)
        ctx.save_for_backward(x, g, b, res if res is not None else None, mean, invstd)
        ctx.cfg = (act, slope, res is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, g, b, res, mean, invstd = ctx.saved_tensors
        act, slope, has_res = ctx.cfg
        dy = dy.contiguous()
        B, H, W, C = x.shape
        M = B * H * W
        nblk = int(lib().jabd_bn_nblk(M, C))
        part = torch.empty((nblk, 2, C), dtype=torch.float32, device=x.device)
        dgamma = torch.empty(C, dtype=torch.float32, device=x.device)
        dbeta = torch.empty_like(dgamma)
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if has_res else None
        call("jabd_bn_act_bwd_f32", dy.data_ptr(), C, 0, x.data_ptr(), C, _p(res), C, M, C,
             mean.data_ptr(), invstd.data_ptr(), g.data_ptr(), b.data_ptr(), ACT[act],
             float(slope), part.data_ptr(), dgamma.data_ptr(), dbeta.data_ptr(), dx.data_ptr(),
             _p(dres), _st())
        return dx, dgamma, dbeta, dres, None, None, None, None, None, None


class DwConvFn(torch.autograd.Function):
    """Depthwise k x k conv (pad k//2), no bias (nets/mobilenetV3.py:105-106)."""

    @staticmethod
    def forward(ctx, x, weight, stride):
        C, _, k, _ = weight.shape
        wt = weight.detach().float().reshape(C, k * k).t().contiguous()
        y, _ = F.dwconv(x, wt, None, k, stride)
        ctx.save_for_backward(x, wt)
        ctx.cfg = (k, stride)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wt = ctx.saved_tensors
        k, stride = ctx.cfg
        dy = dy.contiguous()
        B, H, W, C = x.shape
        OH, OW = dy.shape[1], dy.shape[2]
        pad = k // 2
        dx = torch.empty_like(x)
        call("jabd_dw_dgrad_f32", dy.data_ptr(), wt.data_ptr(), B, H, W, C, OH, OW, k, stride,
             pad, dx.data_ptr(), _st())
        nparts = int(lib().jabd_dw_wgrad_part_floats(B * OH * OW, C, k))
        part = torch.empty(nparts, dtype=torch.float32, device=x.device)
        dw = torch.empty((C, 1, k, k), dtype=torch.float32, device=x.device)
        call("jabd_dw_wgrad_f32", x.data_ptr(), dy.data_ptr(), B, H, W, C, OH, OW, k, stride,
             pad, part.data_ptr(), dw.data_ptr(), _st())
        return dx, dw, None


class NlmFn(torch.autograd.Function):
    """lateral + NLM(nearest(src -> lateral size)) (nets/retinaface_r.py:192-203);
    lateral=None is the standalone NLM.forward(src) (:124-152)."""

    @staticmethod
    def forward(ctx, src, lateral, wq, bq, wk, bk, wv, bv, wW, bW, sizes):
        B, hs, ws, C = src.shape
        ch = wq.shape[0]
        d = lambda t, *s: t.detach().float().reshape(*s).contiguous()  # noqa: E731
        W = (d(wq, ch, C), d(bq, ch), d(wk, ch, C), d(bk, ch), d(wv, ch, C), d(bv, ch),
             d(wW, C, ch), d(bW, C))
        lat = lateral.contiguous() if lateral is not None else None
        out, (q, cx, kp, vp) = F.nlm_fused(src, lat, W, sizes, save=True)
        if lateral is None:
            xup = src
        else:
            _, h, w, _ = lateral.shape
            xup = torch.empty((B, h, w, C), dtype=torch.float32, device=src.device)
            call("jabd_upsample_nearest_f32", src.data_ptr(), B, hs, ws, h, w, C, xup.data_ptr(),
                 _st())
        ctx.save_for_backward(xup, q, cx, kp, vp, *W)
        ctx.cfg = (tuple(sizes), hs, ws, lateral is not None)
        return out

    @staticmethod
    def backward(ctx, dout):
        xup, q, cx, kp, vp, wq, bq, wk, bk, wv, bv, wW, bW = ctx.saved_tensors
        sizes, hs, ws, has_lat = ctx.cfg
        dout = dout.contiguous()
        B, h, w, C = dout.shape
        ch = wq.shape[0]
        S = kp.shape[1]
        dev = dout.device
        nblk = (h * w + 63) // 64  # jabd.h: one partial block per 64 pixels
        dq = torch.empty((B, h, w, ch), dtype=torch.float32, device=dev)
        dxup = torch.empty((B, h, w, C), dtype=torch.float32, device=dev)
        part = torch.empty((B, nblk, S, 2 * ch), dtype=torch.float32, device=dev)
        dk = torch.empty((B, S, ch), dtype=torch.float32, device=dev)
        dv = torch.empty_like(dk)
        call("jabd_nlm_bwd_attn_f32", dout.data_ptr(), B, h, w, C, q.data_ptr(), kp.data_ptr(),
             vp.data_ptr(), S, wW.data_ptr(), wq.data_ptr(), dq.data_ptr(), dxup.data_ptr(),
             part.data_ptr(), dk.data_ptr(), dv.data_ptr(), _st())
        dkv = torch.empty((B, h, w, 2 * ch), dtype=torch.float32, device=dev)
        arr = (ctypes.c_int32 * len(sizes))(*sizes)
        call("jabd_nlm_bwd_proj_f32", dk.data_ptr(), dv.data_ptr(), B, S, arr, len(sizes), h, w,
             C, wk.data_ptr(), wv.data_ptr(), dkv.data_ptr(), dxup.data_ptr(), _st())
        if has_lat:
            dsrc = torch.empty((B, hs, ws, C), dtype=torch.float32, device=dev)
            call("jabd_upsample_nearest_bwd_f32", dxup.data_ptr(), B, h, w, hs, ws, C, 0,
                 dsrc.data_ptr(), _st())
        else:
            dsrc = dxup  # no up-sample: x itself is the source
        # weight gradients = 1x1-conv weight gradients of the saved per-pixel tensors
        ctxv = cx.view(B, h, w, ch)
        dWW = _wgrad(ctxv, dout, torch.empty((C, ch, 1, 1), device=dev), 1, 0)
        dWq = _wgrad(xup, dq, torch.empty((ch, C, 1, 1), device=dev), 1, 0)
        dk_only = torch.empty(dkv.shape[:-1] + (ch,), dtype=torch.float32, device=dev)
        dv_only = torch.empty_like(dk_only)
        kv = dkv.contiguous().view(1, -1, 2 * ch)  # columns are dim 2 of the window
        F.window_copies([(kv, dk_only.view(1, -1, ch), 0.0, 0),
                         (kv, dv_only.view(1, -1, ch), 0.0, ch)])
        dWk = _wgrad(xup, dk_only, torch.empty((ch, C, 1, 1), device=dev), 1, 0)
        dWv = _wgrad(xup, dv_only, torch.empty((ch, C, 1, 1), device=dev), 1, 0)
        g = (dWq, _chan_sum(dq), dWk, _chan_sum(dk_only), dWv, _chan_sum(dv_only), dWW,
             _chan_sum(dout))
        return (dsrc, dout if has_lat else None) + g + (None,)


class UpAddFn(torch.autograd.Function):
    """lateral + F.interpolate(src, size=lateral's, mode='nearest') — the plain
    FPN's merge input (nets/layers.py:106-117)."""

    @staticmethod
    def forward(ctx, src, lateral):
        ctx.src_hw = (src.shape[1], src.shape[2])
        return F.upsample_add(src, lateral.contiguous())

    @staticmethod
    def backward(ctx, dout):
        dout = dout.contiguous()
        B, h, w, C = dout.shape
        hs, ws = ctx.src_hw
        dsrc = torch.empty((B, hs, ws, C), dtype=torch.float32, device=dout.device)
        call("jabd_upsample_nearest_bwd_f32", dout.data_ptr(), B, h, w, hs, ws, C, 0,
             dsrc.data_ptr(), _st())
        return dsrc, dout


class UpsampleFn(torch.autograd.Function):
    """F.interpolate(src, size, mode) on NHWC: nearest, or bicubic with
    align_corners=True (train_mobilenetV3_ecagai.py:270,279)."""

    @staticmethod
    def forward(ctx, src, h, w, mode):
        ctx.cfg = (tuple(src.shape), mode)
        return F.upsample(src.contiguous(), h, w, mode)

    @staticmethod
    def backward(ctx, dout):
        (B, hs, ws, C), mode = ctx.cfg
        dout = dout.contiguous()
        _, h, w, _ = dout.shape
        dsrc = torch.empty((B, hs, ws, C), dtype=torch.float32, device=dout.device)
        if mode == "nearest":
            call("jabd_upsample_nearest_bwd_f32", dout.data_ptr(), B, h, w, hs, ws, C, 0,
                 dsrc.data_ptr(), _st())
        else:
            call("jabd_upsample_bicubic_ac_bwd_f32", dout.data_ptr(), B, hs, ws, C,
                 dsrc.data_ptr(), h, w, _st())
        return dsrc, None, None, None


class Add3Fn(torch.autograd.Function):
    """a + b (+ c) — the NLM residual and the FPN lateral add."""

    @staticmethod
    def forward(ctx, a, b, c):
        ctx.has_c = c is not None
        return F.add3(a.contiguous(), b.contiguous(), c.contiguous() if c is not None else None)

    @staticmethod
    def backward(ctx, d):
        return d, d, (d if ctx.has_c else None)


class NlmAttnFn(torch.autograd.Function):
    """softmax(q . kp^T) . vp (train_mobilenetV3_ecagai.py:216-226) for NLM
    widths other than 4: HIP forward (online softmax) and backward (dq in the
    kernel; dK = dS . q and dV = P . dctx in nlm_attn.hip dkv_part_kernel)."""

    @staticmethod
    def forward(ctx, q, kp, vp):
        q, kp, vp = q.contiguous(), kp.contiguous(), vp.contiguous()
        out, lse = F.nlm_attn(q, kp, vp, save=True)
        ctx.save_for_backward(q, kp, vp, out, lse)
        return out

    @staticmethod
    def backward(ctx, dctx):
        q, kp, vp, out, lse = ctx.saved_tensors
        dctx = dctx.contiguous()
        B, h, w, ch = q.shape
        S = kp.shape[1]
        P = h * w
        dev = q.device
        dq = torch.empty_like(q)
        pm = torch.empty((B, S, P), dtype=torch.float32, device=dev)
        dsm = torch.empty_like(pm)
        call("jabd_nlm_attn_bwd_f32", q.data_ptr(), kp.data_ptr(), vp.data_ptr(), out.data_ptr(),
             lse.data_ptr(), dctx.data_ptr(), B, P, S, ch, dq.data_ptr(), pm.data_ptr(),
             dsm.data_ptr(), _st())
        # [S x P] . [P x ch] per image on the MFMA, chunks over P summed in order
        dk = torch.empty_like(kp)
        dv = torch.empty_like(vp)
        nws = int(lib().jabd_nlm_attn_dkv_ws_floats(B, P, S, ch))
        ws = torch.empty(nws, dtype=torch.float32, device=dev)
        call("jabd_nlm_attn_dkv_f32", dsm.data_ptr(), pm.data_ptr(), q.data_ptr(),
             dctx.data_ptr(), B, P, S, ch, ws.data_ptr(), nws, dk.data_ptr(), dv.data_ptr(), _st())
        return dq, dk, dv


class SshTailFn(torch.autograd.Function):
    """relu(cat(BN(a), BN(b), BN(c))) of SSH (nets/layers.py:56-68)."""

    @staticmethod
    def forward(ctx, a, b, c, ga, ba, gb, bb, gc, bc, stats):
        outs = []
        B, H, W, _ = a.shape
        Ctot = a.shape[3] + b.shape[3] + c.shape[3]
        y = torch.empty((B, H, W, Ctot), dtype=torch.float32, device=a.device)
        saved = []
        c0 = 0
        for x, g, bt, (rm, rv, mom, eps) in zip((a, b, c), (ga, gb, gc), (ba, bb, bc), stats):
            C = x.shape[3]
            M = B * H * W
            nblk = int(lib().jabd_bn_nblk(M, C))
            part = torch.empty((nblk, 2, C), dtype=torch.float32, device=x.device)
            mean = torch.empty(C, dtype=torch.float32, device=x.device)
            invstd = torch.empty_like(mean)
            call("jabd_bn_stats_f32", x.data_ptr(), C, M, C, part.data_ptr(), mean.data_ptr(),
                 invstd.data_ptr(), _p(rm), _p(rv), float(mom), float(eps), _st())
            F.tap("stats", "bn_stats", x, mean, invstd, eps)
            gg, bb_ = g.detach().contiguous(), bt.detach().contiguous()
            call("jabd_bn_act_fwd_f32", x.data_ptr(), C, M, C, mean.data_ptr(),
                 invstd.data_ptr(), gg.data_ptr(), bb_.data_ptr(), None, C, ACT["relu"], 0.0,
                 y.data_ptr(), Ctot, c0, _st())
            saved += [x, gg, bb_, mean, invstd]
            outs.append(c0)
            c0 += C
        F.tap("ssh", [saved[5 * i:5 * i + 5] for i in range(3)])
        ctx.save_for_backward(*saved)
        ctx.offs = outs
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        sv = ctx.saved_tensors
        res = []
        Ctot = dy.shape[3]
        for i in range(3):
            x, g, b, mean, invstd = sv[5 * i:5 * i + 5]
            B, H, W, C = x.shape
            M = B * H * W
            nblk = int(lib().jabd_bn_nblk(M, C))
            part = torch.empty((nblk, 2, C), dtype=torch.float32, device=x.device)
            dg = torch.empty(C, dtype=torch.float32, device=x.device)
            db = torch.empty_like(dg)
            dx = torch.empty_like(x)
            call("jabd_bn_act_bwd_f32", dy.data_ptr(), Ctot, ctx.offs[i], x.data_ptr(), C, None,
                 C, M, C, mean.data_ptr(), invstd.data_ptr(), g.data_ptr(), b.data_ptr(),
                 ACT["relu"], 0.0, part.data_ptr(), dg.data_ptr(), db.data_ptr(), dx.data_ptr(),
                 None, _st())
            res.append((dx, dg, db))
        (da, dga, dba), (dbx, dgb, dbb), (dc, dgc, dbc) = res
        return da, dbx, dc, dga, dba, dgb, dbb, dgc, dbc, None


class HeadsFn(torch.autograd.Function):
    """Bbox/Class/Landmark 1x1 heads of the 3 levels -> (loc, conf, landm) logits."""

    @staticmethod
    def forward(ctx, f1, f2, f3, cidx, *wb):
        """cidx: per level None, or the (half, q, qp) layout of a feature
        tensor whose two q-channel branches are zero-padded to qp channels
        (ssh_train(padded_out=True))."""
        feats = (f1, f2, f3)
        B = f1.shape[0]
        A = sum(2 * f.shape[1] * f.shape[2] for f in feats)
        dev = f1.device
        loc = torch.empty((B, A, 4), dtype=torch.float32, device=dev)
        conf = torch.empty((B, A, 2), dtype=torch.float32, device=dev)
        landm = torch.empty((B, A, 10), dtype=torch.float32, device=dev)
        a_off = 0
        cat = []
        for i, f in enumerate(feats):
            ws = [t.detach() for t in wb[6 * i:6 * i + 6]]  # Wb, bb, Wc, bc, Wl, bl
            C = ws[0].shape[1]
            Cf = f.shape[3]
            half, q, qp = cidx[i] if cidx[i] is not None else (C, 0, 0)
            wt = torch.empty((32, Cf), dtype=torch.float32, device=dev)
            bs = torch.empty(32, dtype=torch.float32, device=dev)
            call("jabd_heads_wpack_f32", ws[0].data_ptr(), ws[2].data_ptr(), ws[4].data_ptr(),
                 ws[1].data_ptr(), ws[3].data_ptr(), ws[5].data_ptr(), C, half, q, qp,
                 wt.data_ptr(), Cf, bs.data_ptr(), 0, _st())
            F.heads(f, wt, bs, loc, conf, landm, a_off, softmax=False)
            cat.append(wt)
            a_off += 2 * f.shape[1] * f.shape[2]
        ctx.save_for_backward(f1, f2, f3, *cat)
        ctx.cidx = cidx
        ctx.cs = [wb[6 * i].shape[1] for i in range(3)]
        return loc, conf, landm

    @staticmethod
    def backward(ctx, gl, gc, glm):
        f1, f2, f3, w1, w2, w3 = ctx.saved_tensors
        dev = f1.device
        B = f1.shape[0]
        A = sum(2 * f.shape[1] * f.shape[2] for f in (f1, f2, f3))
        zero = None
        if gl is None or gc is None or glm is None:
            zero = torch.empty((B, A, 10), dtype=torch.float32, device=dev)
            F.window_copies([(None, zero, 0.0)])
        gl = gl.contiguous() if gl is not None else zero[..., :4].contiguous()
        gc = gc.contiguous() if gc is not None else zero[..., :2].contiguous()
        glm = glm.contiguous() if glm is not None else zero
        a_off = 0
        dfs, dws = [], []
        for i, (f, wt) in enumerate(zip((f1, f2, f3), (w1, w2, w3))):
            _, h, w, Cf = f.shape
            dout = torch.empty((B, h, w, 32), dtype=torch.float32, device=dev)
            call("jabd_heads_gather_f32", gl.data_ptr(), gc.data_ptr(), glm.data_ptr(), B, A,
                 a_off, h * w, dout.data_ptr(), _st())
            wconv = wt.view(32, Cf, 1, 1)
            dfs.append(_dgrad(dout, wconv, 1, 0, h, w))
            dW = _wgrad(f, dout, wconv, 1, 0).view(32, Cf)
            C = ctx.cs[i]
            half, q, qp = ctx.cidx[i] if ctx.cidx[i] is not None else (C, 0, 0)
            g3 = [torch.empty((r, C, 1, 1), dtype=torch.float32, device=dev) for r in (8, 4, 20)]
            call("jabd_heads_wpack_f32", g3[0].data_ptr(), g3[1].data_ptr(), g3[2].data_ptr(),
                 None, None, None, C, half, q, qp, dW.data_ptr(), Cf, None, 1, _st())
            db = _chan_sum(dout)
            dws += [g3[0], db[:8], g3[1], db[8:12], g3[2], db[12:]]
            a_off += 2 * h * w
        return tuple(dfs) + (None,) + tuple(dws)


class MaxPoolFn(torch.autograd.Function):
    """3x3/2/1 max-pool of the R50 stem; the forward keeps the argmax window
    positions (uint8) so the backward is a gather of idx + dy."""

    @staticmethod
    def forward(ctx, x):
        B, H, W, C = x.shape
        OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        x = x.contiguous()
        y = torch.empty((B, OH, OW, C), dtype=torch.float32, device=x.device)
        idx = torch.empty((B, OH, OW, C), dtype=torch.uint8, device=x.device)
        call("jabd_maxpool_idx_nhwc_f32", x.data_ptr(), B, H, W, C, 3, 2, 1, y.data_ptr(),
             idx.data_ptr(), _st())
        F.tap("maxpool", x)
        ctx.save_for_backward(idx)
        ctx.shape = (B, H, W, C)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        dy = dy.contiguous()
        B, H, W, C = ctx.shape
        dx = torch.empty((B, H, W, C), dtype=torch.float32, device=dy.device)
        call("jabd_maxpool_bwd_idx_f32", idx.data_ptr(), dy.data_ptr(), B, H, W, C, 3, 2, 1,
             dx.data_ptr(), _st())
        return dx


# ----------------------------------------------------------------------------- graph helpers
def _pad_to4(c):
    return (c + 3) // 4 * 4


def bn_act(x, bn, act="none", slope=0.0, res=None):
    """BatchNorm2d module (training) + activation, padded channels allowed."""
    C = x.shape[3]
    g, b = bn.weight, bn.bias
    rm, rv = bn.running_mean, bn.running_var
    if C != g.shape[0]:  # zero-padded channels (10 -> 12): pad params/buffers
        g, b, rm_p, rv_p = _padded([(g, (C,), 0.0), (b, (C,), 0.0), (rm, (C,), 0.0),
                                    (rv, (C,), 1.0)])
        y = BnActFn.apply(x, g, b, res, rm_p, rv_p, act, slope, bn.momentum, bn.eps)
        with torch.no_grad():
            F.window_copies([(rm_p, rm, 0.0), (rv_p, rv, 0.0)])
    else:
        y = BnActFn.apply(x, g, b, res, rm, rv, act, slope, bn.momentum, bn.eps)
    _count_batch(bn)
    return y


# num_batches_tracked increments of one train_forward, applied as one
# multi-tensor add at its end (75 one-element kernels otherwise).  Per thread:
# nn.DataParallel runs the replicas' forwards on concurrent threads.
_NBT = threading.local()


def _nbt_stack():
    st = getattr(_NBT, "stack", None)
    if st is None:
        st = _NBT.stack = []
    return st


def _count_batch(bn):
    t = bn.num_batches_tracked
    if t is None:
        return
    st = _nbt_stack()
    if st:
        st[-1].append(t)
    else:
        t.add_(1)


class _BatchCounts:
    def __enter__(self):
        _nbt_stack().append([])

    def __exit__(self, *exc):
        ts = _nbt_stack().pop()
        if ts and exc[0] is None:
            torch._foreach_add_(ts, 1)


class PadFn(torch.autograd.Function):
    """Zero-pad several tensors along dims 0 / 1 in one launch (conv weights
    [Cout][Cin][..] and BN vectors [C] of the 10-channel SSH branches ->
    12 channels); the backward crops the gradients back in one launch.
    spec: per tensor (padded shape, fill)."""

    @staticmethod
    def forward(ctx, spec, *ts):
        ctx.set_materialize_grads(False)
        outs, items = [], []
        for t, (shape, fill) in zip(ts, spec):
            t = t.detach()
            if not t.is_contiguous():
                t = t.contiguous()
            o = torch.empty(shape, dtype=torch.float32, device=t.device)
            items.append((t, o, fill))
            outs.append(o)
        F.window_copies(items)
        ctx.shapes = [tuple(t.shape) for t in ts]
        nd = [o for t, o in zip(ts, outs) if not t.requires_grad]
        if nd:
            ctx.mark_non_differentiable(*nd)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        items, res = [], []
        for g, shape in zip(gs, ctx.shapes):
            if g is None:
                res.append(None)
                continue
            o = torch.empty(shape, dtype=torch.float32, device=g.device)
            items.append((g if g.is_contiguous() else g.contiguous(), o, 0.0))
            res.append(o)
        F.window_copies(items)
        return (None,) + tuple(res)


class ForkFn(torch.autograd.Function):
    """n aliases of one tensor for n consumers: the backward sums their
    gradients in one HIP launch (jabd_sum_multi_f32) instead of the autograd
    engine's pairwise ATen adds."""

    @staticmethod
    def forward(ctx, x, n):
        ctx.set_materialize_grads(False)
        return tuple(x.view_as(x) for _ in range(n))

    @staticmethod
    def backward(ctx, *gs):
        gs = [g if g.is_contiguous() else g.contiguous() for g in gs if g is not None]
        if not gs:
            return None, None
        if len(gs) == 1:
            return gs[0], None
        out = torch.empty_like(gs[0], memory_format=torch.contiguous_format)
        ptrs = (ctypes.c_void_p * len(gs))(*[g.data_ptr() for g in gs])
        call("jabd_sum_multi_f32", len(gs), ptrs, out.numel(), out.data_ptr(), _st())
        return out, None


def fork(x, n):
    """n autograd aliases of x (ForkFn); x itself when it needs no gradient."""
    if not x.requires_grad or not torch.is_grad_enabled():
        return (x,) * n
    return ForkFn.apply(x, n)


def _padded(spec_ts):
    """[(tensor, padded shape, fill)] -> padded tensors (one PadFn launch)."""
    return PadFn.apply(tuple((tuple(shape), fill) for _, shape, fill in spec_ts),
                       *[t for t, _, _ in spec_ts])


def _padw(weight, cout=None, cin=None):
    """Zero-pad a conv weight's out/in channels (autograd-tracked, one launch)."""
    co = max(cout or 0, weight.shape[0])
    ci = max(cin or 0, weight.shape[1])
    if (co, ci) == tuple(weight.shape[:2]):
        return weight
    return _padded([(weight, (co, ci) + tuple(weight.shape[2:]), 0.0)])[0]


def conv(x, m, stride=1, pad=0, nchw_in=False):
    return ConvFn.apply(x, m.weight, m.bias, stride, pad, nchw_in)


# ----------------------------------------------------------------------------- fused block
def _bn_stats(x, bn):
    """Batch statistics (mean, invstd) of NHWC x for bn (jabd_bn_stats_f32;
    running buffers updated)."""
    B, H, W, C = x.shape
    M = B * H * W
    nblk = int(lib().jabd_bn_nblk(M, C))
    part = torch.empty((nblk, 2, C), dtype=torch.float32, device=x.device)
    mean = torch.empty(C, dtype=torch.float32, device=x.device)
    invstd = torch.empty_like(mean)
    call("jabd_bn_stats_f32", x.data_ptr(), C, M, C, part.data_ptr(), mean.data_ptr(),
         invstd.data_ptr(), bn.running_mean.data_ptr(), bn.running_var.data_ptr(),
         float(bn.momentum), float(bn.eps), _st())
    F.tap("stats", "bn_stats", x, mean, invstd, bn.eps)
    return mean, invstd


def _bn_fwd(x, bn, act, slope=0.0, res=None, sums=False, stats=None):
    """Batch-stat BN (+res) + act of NHWC x; running buffers updated in place.
    Returns (y, (gamma, beta, mean, invstd)); sums=True adds the per-image
    channel-sum partials of y ([B, nblk, C], written by the apply pass) or
    None when the map size does not fit its row blocks.  stats = (mean,
    invstd) already computed by x's producer (running buffers updated there)."""
    B, H, W, C = x.shape
    M = B * H * W
    if stats is not None:
        mean, invstd = stats
    else:
        nblk = int(lib().jabd_bn_nblk(M, C))
        part = torch.empty((nblk, 2, C), dtype=torch.float32, device=x.device)
        mean = torch.empty(C, dtype=torch.float32, device=x.device)
        invstd = torch.empty_like(mean)
        call("jabd_bn_stats_f32", x.data_ptr(), C, M, C, part.data_ptr(), mean.data_ptr(),
             invstd.data_ptr(), bn.running_mean.data_ptr(), bn.running_var.data_ptr(),
             float(bn.momentum), float(bn.eps), _st())
        F.tap("stats", "bn_stats", x, mean, invstd, bn.eps)
    g = bn.weight.detach()
    b = bn.bias.detach()
    y = torch.empty_like(x)
    nsum = int(lib().jabd_bn_sum_nblk(H * W, C)) if sums and ECA_SUMS and res is None and \
        x.is_contiguous() else 0
    if nsum:
        psum = torch.empty((B, nsum, C), dtype=torch.float32, device=x.device)
        call("jabd_bn_act_fwd_sum_f32", x.data_ptr(), M, C, mean.data_ptr(), invstd.data_ptr(),
             g.data_ptr(), b.data_ptr(), ACT[act], float(slope), y.data_ptr(), H * W,
             psum.data_ptr(), _st())
    else:
        psum = None
        call("jabd_bn_act_fwd_f32", x.data_ptr(), C, M, C, mean.data_ptr(), invstd.data_ptr(),
             g.data_ptr(), b.data_ptr(), _p(res), C, ACT[act], float(slope), y.data_ptr(), C, 0,
             _st())
    _count_batch(bn)
    if act != "none":
        F.tap("bn", act, slope, x, mean, invstd, g, b, res)
    if sums:
        return y, (g, b, mean, invstd), psum
    return y, (g, b, mean, invstd)


def _bn_bwd(dy, x, st, act, slope=0.0, res=None, want_dres=False, dys=None, dya=None):
    """Backward of _bn_fwd: (dx, dgamma, dbeta, dres); dys/dya: the per-(image,
    channel) map of dy (jabd_bn_act_bwd_ex_f32)."""
    g, b, mean, invstd = st
    B, H, W, C = x.shape
    M = B * H * W
    nblk = int(lib().jabd_bn_nblk(M, C))
    part = torch.empty((nblk, 2, C), dtype=torch.float32, device=x.device)
    dgamma = torch.empty(C, dtype=torch.float32, device=x.device)
    dbeta = torch.empty_like(dgamma)
    dx = torch.empty_like(x)
    dres = torch.empty_like(x) if want_dres else None
    call("jabd_bn_act_bwd_ex_f32", dy.data_ptr(), C, 0, x.data_ptr(), C, _p(res), C, M, C,
         mean.data_ptr(), invstd.data_ptr(), g.data_ptr(), b.data_ptr(), ACT[act], float(slope),
         _p(dys), _p(dya), H * W if dys is not None else 0, part.data_ptr(), dgamma.data_ptr(),
         dbeta.data_ptr(), dx.data_ptr(), _p(dres), _st())
    return dx, dgamma, dbeta, dres


def _conv_fwd(x, weight, bias=None, stride=1, pad=0, ascale=None):
    pk = _packed(weight, transposed=False)
    B, H, W, _ = x.shape
    OH = (H + 2 * pad - pk.KH) // stride + 1
    OW = (W + 2 * pad - pk.KW) // stride + 1
    y = torch.empty((B, OH, OW, pk.Cout), dtype=torch.float32, device=x.device)
    a = _conv_args(x, pk, y, stride, pad, ascale=ascale)
    if bias is not None:
        bb = bias.detach()
        a.bias = bb.data_ptr()
    call("jabd_conv2d_nhwc_f32", ctypes.byref(a), _st())
    return y


def _conv_fwd_bn_stats(x, weight, bn):
    """Bias-free 1x1 _conv_fwd whose streaming kernel also takes the batch
    statistics of its output for the following BatchNorm
    (jabd_conv1x1_bn_stats_f32 + jabd_bn_stats_final_f32; running buffers
    updated).  Returns (y, (mean, invstd)), or (y, None) when the statistics
    form does not serve the layer (the caller's _bn_fwd then takes them).
    Layers the streaming form does not take (Cout > 80) go to the 32x32
    GEMM's statistics form (_conv_fwd_stats)."""
    pk = _packed(weight, transposed=False)
    B, H, W, _ = x.shape
    y = torch.empty((B, H, W, pk.Cout), dtype=torch.float32, device=x.device)
    a = _conv_args(x, pk, y, 1, 0)
    nblk = int(lib().jabd_conv1x1_bn_stats_nblk(ctypes.byref(a))) if pk.KH == 1 else 0
    if nblk <= 0:
        return _conv_fwd_stats(x, weight, bn)
    C = pk.Cout
    part = torch.empty((nblk, 2, C), dtype=torch.float32, device=x.device)
    shift = torch.empty(C, dtype=torch.float32, device=x.device)
    call("jabd_conv1x1_bn_stats_f32", ctypes.byref(a), part.data_ptr(), nblk, shift.data_ptr(),
         _st())
    mean = torch.empty(C, dtype=torch.float32, device=x.device)
    invstd = torch.empty_like(mean)
    call("jabd_bn_stats_final_f32", shift.data_ptr(), part.data_ptr(), nblk, B * H * W, C,
         mean.data_ptr(), invstd.data_ptr(), bn.running_mean.data_ptr(),
         bn.running_var.data_ptr(), float(bn.momentum), float(bn.eps), _st())
    F.tap("stats", "conv1x1_stream", y, mean, invstd, bn.eps)
    return y, (mean, invstd)


def _conv_fwd_stats(x, weight, bn, stride=1, pad=0):
    """Bias-free _conv_fwd on the 32x32 GEMM whose epilogue also takes the
    batch statistics of its output for the following BatchNorm
    (jabd_conv_bn_stats_f32: per-32-pixel-tile rows, combined in fp64 in a
    fixed order; running buffers updated).  Returns (y, (mean, invstd)), or
    (y, None) when the form does not serve the layer (the caller's _bn_fwd
    then takes the statistics)."""
    pk = _packed(weight, transposed=False)
    B, H, W, _ = x.shape
    OH = (H + 2 * pad - pk.KH) // stride + 1
    OW = (W + 2 * pad - pk.KW) // stride + 1
    y = torch.empty((B, OH, OW, pk.Cout), dtype=torch.float32, device=x.device)
    a = _conv_args(x, pk, y, stride, pad)
    nf = int(lib().jabd_conv_bn_stats_part_floats(ctypes.byref(a)))
    if nf <= 0:
        call("jabd_conv2d_nhwc_f32", ctypes.byref(a), _st())
        return y, None
    part = torch.empty(nf, dtype=torch.float32, device=x.device)
    mean = torch.empty(pk.Cout, dtype=torch.float32, device=x.device)
    invstd = torch.empty_like(mean)
    call("jabd_conv_bn_stats_f32", ctypes.byref(a), part.data_ptr(), nf, mean.data_ptr(),
         invstd.data_ptr(), bn.running_mean.data_ptr(), bn.running_var.data_ptr(),
         float(bn.momentum), float(bn.eps), _st())
    F.tap("stats", "conv32", y, mean, invstd, bn.eps)
    return y, (mean, invstd)


def _dgrad_bn_sums(dy, weight, stride, pad, H, W, x, st, act):
    """_dgrad whose output is the dy of the BatchNorm (+ act) st of x: the
    32x32 GEMM's epilogue also takes that BatchNorm backward's sums
    (jabd_conv_bn_bwd_sums_f32).  Returns (dx, part) — part None when the
    form does not serve the conv (then _bn_bwd takes the sums itself)."""
    pk = _packed(weight, transposed=True)
    B = dy.shape[0]
    dx = torch.empty((B, H, W, pk.Cout), dtype=torch.float32, device=dy.device)
    plain = pk.KH == 1 and pk.KW == 1 and stride == 1 and pad == 0
    a = _conv_args(dy, pk, dx, stride, pad, tconv=not plain, OH=H, OW=W)
    nf = int(lib().jabd_conv_bn_bwd_part_floats(ctypes.byref(a))) if BN_BWD_EPI else 0
    if nf <= 0 or not x.is_contiguous():
        call("jabd_conv2d_nhwc_f32", ctypes.byref(a), _st())
        return dx, None
    g, b, mean, invstd = st
    part = torch.empty(nf, dtype=torch.float32, device=dy.device)
    call("jabd_conv_bn_bwd_sums_f32", ctypes.byref(a), x.data_ptr(), x.shape[3], mean.data_ptr(),
         invstd.data_ptr(), g.data_ptr(), b.data_ptr(), ACT[act], 0.0, part.data_ptr(), nf,
         _st())
    return dx, part


def _bn_bwd_rows(dy, x, st, act, part):
    """_bn_bwd (no residual) from the sums _dgrad_bn_sums took."""
    g, b, mean, invstd = st
    B, H, W, C = x.shape
    dgamma = torch.empty(C, dtype=torch.float32, device=x.device)
    dbeta = torch.empty_like(dgamma)
    dx = torch.empty_like(x)
    call("jabd_bn_act_bwd_rows_f32", part.data_ptr(), dy.data_ptr(), x.data_ptr(), B * H * W, C,
         mean.data_ptr(), invstd.data_ptr(), g.data_ptr(), b.data_ptr(), ACT[act], 0.0,
         dgamma.data_ptr(), dbeta.data_ptr(), dx.data_ptr(), _st())
    return dx, dgamma, dbeta, None


def _dgrad_1x1_res(dy, weight, res):
    """dx = dgrad of a 1x1 / stride-1 conv, + res added in the GEMM epilogue."""
    pk = _packed(weight, transposed=True)
    B, H, W, _ = dy.shape
    dx = torch.empty((B, H, W, pk.Cout), dtype=torch.float32, device=dy.device)
    a = _conv_args(dy, pk, dx, 1, 0)
    if res is not None:
        a.res, a.res_bs, a.res_ps, a.res_c0 = res.data_ptr(), res.stride(0), res.shape[3], 0
    call("jabd_conv2d_nhwc_f32", ctypes.byref(a), _st())
    return dx


def _dgrad_1x1_res_bn3(dy, weight, res, out, x3, st3):
    """_dgrad_1x1_res whose output is the dout of the previous bottleneck's
    out = relu(bn3(x3) + identity): the GEMM writes dz = (dgrad + res) *
    [out > 0] and bn3's backward sums (jabd_conv_bn_bwd_sums_res_f32).
    Returns (dz, part), or (dx, None) — the plain data gradient — when the
    form does not serve the conv."""
    pk = _packed(weight, transposed=True)
    B, H, W, _ = dy.shape
    dx = torch.empty((B, H, W, pk.Cout), dtype=torch.float32, device=dy.device)
    a = _conv_args(dy, pk, dx, 1, 0)
    nf = int(lib().jabd_conv_bn_bwd_part_floats(ctypes.byref(a)))
    if res is not None:
        a.res, a.res_bs, a.res_ps, a.res_c0 = res.data_ptr(), res.stride(0), res.shape[3], 0
    if nf <= 0 or not (out.is_contiguous() and x3.is_contiguous() and
                       (res is None or res.is_contiguous())):
        call("jabd_conv2d_nhwc_f32", ctypes.byref(a), _st())
        return dx, None
    _, _, mean, invstd = st3
    part = torch.empty(nf, dtype=torch.float32, device=dy.device)
    call("jabd_conv_bn_bwd_sums_res_f32", ctypes.byref(a), x3.data_ptr(), x3.shape[3],
         out.data_ptr(), out.shape[3], mean.data_ptr(), invstd.data_ptr(), part.data_ptr(), nf,
         _st())
    return dx, part


def _dw_fwd(x, weight, stride):
    C, _, k, _ = weight.shape
    wt = F.transpose(weight.detach().reshape(C, k * k))  # tap-major [k*k][C]
    y, _ = F.dwconv(x, wt, None, k, stride)
    return y, wt


def _dw_fwd_bn_stats(x, weight, stride, bn, bnin=None):
    """_dw_fwd whose kernel also takes the batch statistics of its output for
    the following BatchNorm (jabd_dwconv_stats_f32 + jabd_bn_stats_final_f32;
    running buffers updated).  bnin = ((gamma, beta, mean, invstd), act): x
    is the pre-BN tensor and the kernel convolves act(bn(x)), applied on load
    (jabd_dwconv_bnin_stats_f32).  Returns (y, wt, (mean, invstd))."""
    C, _, k, _ = weight.shape
    wt = F.transpose(weight.detach().reshape(C, k * k))
    B, H, W, _ = x.shape
    pad = k // 2
    OH = (H + 2 * pad - k) // stride + 1
    OW = (W + 2 * pad - k) // stride + 1
    y = torch.empty((B, OH, OW, C), dtype=torch.float32, device=x.device)
    a = F.DwArgs()
    a.x, a.x_bs, a.x_ps = x.data_ptr(), x.stride(0), C
    a.B, a.H, a.W, a.C = B, H, W, C
    a.w, a.bias = wt.data_ptr(), None
    a.y, a.y_bs, a.y_ps = y.data_ptr(), y.stride(0), C
    a.OH, a.OW, a.k, a.stride, a.pad, a.act = OH, OW, k, stride, pad, ACT["none"]
    nblk = int(lib().jabd_dwconv_stats_nblk(B, OH, OW, C))
    part = torch.empty((nblk, 2, C), dtype=torch.float32, device=x.device)
    shift = torch.empty(C, dtype=torch.float32, device=x.device)
    if bnin is None:
        call("jabd_dwconv_stats_f32", ctypes.byref(a), part.data_ptr(), shift.data_ptr(), _st())
    else:
        (g1, b1, m1, i1), act1 = bnin
        call("jabd_dwconv_bnin_stats_f32", ctypes.byref(a), m1.data_ptr(), i1.data_ptr(),
             g1.data_ptr(), b1.data_ptr(), ACT[act1], 0.0, part.data_ptr(), shift.data_ptr(),
             _st())
    mean = torch.empty(C, dtype=torch.float32, device=x.device)
    invstd = torch.empty_like(mean)
    call("jabd_bn_stats_final_f32", shift.data_ptr(), part.data_ptr(), nblk, B * OH * OW, C,
         mean.data_ptr(), invstd.data_ptr(), bn.running_mean.data_ptr(),
         bn.running_var.data_ptr(), float(bn.momentum), float(bn.eps), _st())
    F.tap("stats", "dw" if bnin is None else "dw_bnin", y, mean, invstd, bn.eps)
    return y, wt, (mean, invstd)


def _dw_bwd(dy, x, wt, k, stride, want_dx=True, bnin=None):
    """bnin: as in _dw_fwd_bn_stats (x pre-BN; the weight gradient's taps
    recomputed as act(bn(x)), jabd_dw_wgrad_bnin_f32; needs want_dx=False)."""
    B, H, W, C = x.shape
    OH, OW = dy.shape[1], dy.shape[2]
    pad = k // 2
    dx = None
    if want_dx:
        assert bnin is None
        dx = torch.empty_like(x)
        call("jabd_dw_dgrad_f32", dy.data_ptr(), wt.data_ptr(), B, H, W, C, OH, OW, k, stride,
             pad, dx.data_ptr(), _st())
    nparts = int(lib().jabd_dw_wgrad_part_floats(B * OH * OW, C, k))
    part = torch.empty(nparts, dtype=torch.float32, device=x.device)
    dw = torch.empty((C, 1, k, k), dtype=torch.float32, device=x.device)
    if bnin is None:
        call("jabd_dw_wgrad_f32", x.data_ptr(), dy.data_ptr(), B, H, W, C, OH, OW, k, stride, pad,
             part.data_ptr(), dw.data_ptr(), _st())
    else:
        (g1, b1, m1, i1), act1 = bnin
        call("jabd_dw_wgrad_bnin_f32", x.data_ptr(), dy.data_ptr(), B, H, W, C, OH, OW, k, stride,
             pad, m1.data_ptr(), i1.data_ptr(), g1.data_ptr(), b1.data_ptr(), ACT[act1], 0.0,
             part.data_ptr(), dw.data_ptr(), _st())
    return dx, dw


def _dw_bn_bwd(dy, x, wt, k, stride, x_bn, st, act):
    """Backward of d = dwconv(act(bn(x_bn))) with x = act(bn(x_bn)): the
    depthwise data gradient carries bn's backward partials
    (jabd_dw_dgrad_bn_bwd_f32).  x None: it was never stored (BN-input
    forward) and the weight gradient recomputes it from x_bn.  Returns
    (dx_bn, dgamma, dbeta, dW)."""
    g, b, mean, invstd = st
    B, H, W, C = x_bn.shape
    OH, OW = dy.shape[1], dy.shape[2]
    nparts = int(lib().jabd_dw_dgrad_bn_part_floats(B, H, W, C))
    part = torch.empty(nparts, dtype=torch.float32, device=x_bn.device)
    dgamma = torch.empty(C, dtype=torch.float32, device=x_bn.device)
    dbeta = torch.empty_like(dgamma)
    # stride 2 only: there dy is a quarter of de; at stride 1 the kernel is
    # not HBM-bound and the second depthwise pass costs more than de's
    # write + read (r03 C4 profile)
    dz = None if DGBN_RECOMPUTE and stride == 2 else torch.empty_like(x_bn)
    dx = torch.empty_like(x_bn)
    call("jabd_dw_dgrad_bn_bwd_f32", dy.data_ptr(), wt.data_ptr(), B, H, W, C, OH, OW, k, stride,
         k // 2, x_bn.data_ptr(), mean.data_ptr(), invstd.data_ptr(), g.data_ptr(), b.data_ptr(),
         ACT[act], 0.0, part.data_ptr(), dgamma.data_ptr(), dbeta.data_ptr(), _p(dz),
         dx.data_ptr(), _st())
    if x is None:
        _, dw = _dw_bwd(dy, x_bn, wt, k, stride, want_dx=False, bnin=(st, act))
    else:
        _, dw = _dw_bwd(dy, x, wt, k, stride, want_dx=False)
    return dx, dgamma, dbeta, dw


class MNv3BlockFn(torch.autograd.Function):
    """One Block_eca (nets/mobilenetV3.py:94-150) forward and backward as a
    single autograd node, so the backward can fuse what per-op nodes cannot:

      * the ECA gate's backward: the consumer conv's data gradient da, the
        per-image partials sum(da * d) and the gate backward give
        dd = da * scale + dmean/HW, which is applied inside BN2's backward
        as its dy map (jabd_bn_act_bwd_ex_f32) — no dx pass over d;
      * the residual: the skip branch's input gradient is added in the
        epilogue of conv1's data-gradient GEMM — no autograd add pass.

    Inputs: the block (config + buffers), s, then the parameters in the
    order of _block_params(blk)."""

    @staticmethod
    def forward(ctx, blk, s, *params):
        act = blk.act_name
        k, stride = blk.kernel_size, blk.stride
        if DW_BN_FUSE:
            e_pre, bst1 = _conv_fwd_bn_stats(s, blk.conv1.weight, blk.bn1)
        else:
            e_pre, bst1 = _conv_fwd(s, blk.conv1.weight), None
        if DW_BN_FUSE and DW_BNIN and k == 3 and (stride == 2 or DW_BNIN_S1):
            # bn1 + act applied on conv2's loads: e is never written
            if bst1 is None:
                bst1 = _bn_stats(e_pre, blk.bn1)
            st1 = (blk.bn1.weight.detach(), blk.bn1.bias.detach()) + tuple(bst1)
            _count_batch(blk.bn1)
            F.tap("bn", act, 0.0, e_pre, st1[2], st1[3], st1[0], st1[1], None)
            e = None
            d_pre, wt2, bst2 = _dw_fwd_bn_stats(e_pre, blk.conv2.weight, stride, blk.bn2,
                                                bnin=(st1, act))
            d, st2, psum = _bn_fwd(d_pre, blk.bn2, act, sums=True, stats=bst2)
        elif DW_BN_FUSE:
            e, st1 = _bn_fwd(e_pre, blk.bn1, act, stats=bst1)
            d_pre, wt2, bst2 = _dw_fwd_bn_stats(e, blk.conv2.weight, stride, blk.bn2)
            d, st2, psum = _bn_fwd(d_pre, blk.bn2, act, sums=True, stats=bst2)
        else:
            e, st1 = _bn_fwd(e_pre, blk.bn1, act, stats=bst1)
            d_pre, wt2 = _dw_fwd(e, blk.conv2.weight, stride)
            d, st2, psum = _bn_fwd(d_pre, blk.bn2, act, sums=True)
        B, OH, OW, E = d.shape
        w1 = blk.eca.conv.weight.detach().reshape(-1).float().contiguous()
        if psum is None:
            psum = F.channel_sums(d)
        scale, mean = F.eca_gate(psum, OH * OW, w1, "hsigmoid", return_mean=True)
        F.tap("eca", "hsigmoid", mean, w1)
        p = _conv_fwd(d, blk.conv3.weight, ascale=scale)
        sk = blk.skip
        saved_skip = ()
        if sk is None:
            kind, res = "identity", s
        elif stride == 1:
            kind = "concat"
            t_pre = _conv_fwd(s, sk[0].weight, sk[0].bias)
            res, sts0 = _bn_fwd(t_pre, sk[1], "none")
            saved_skip = (t_pre,)
        elif len(sk) == 4:
            kind = "dw_concat"
            u_pre, wts = _dw_fwd(s, sk[0].weight, 2)
            u, sts0 = _bn_fwd(u_pre, sk[1], "none")
            t_pre = _conv_fwd(u, sk[2].weight, sk[2].bias)
            res, sts2 = _bn_fwd(t_pre, sk[3], "none")
            saved_skip = (u_pre, u, t_pre, wts)
        else:
            kind = "dw_residual"
            u_pre, wts = _dw_fwd(s, sk[0].weight, 2)
            res, sts0 = _bn_fwd(u_pre, sk[1], "none")
            saved_skip = (u_pre, wts)
        out, st3 = _bn_fwd(p, blk.bn3, act, res=res)
        ctx.blk, ctx.kind = blk, kind
        ctx.stats = [st1, st2, st3] + ([sts0] if kind != "identity" else []) + \
            ([sts2] if kind == "dw_concat" else [])
        ctx.save_for_backward(s, e_pre, e, d_pre, d, p, res, scale, mean, wt2, *saved_skip)
        return out

    @staticmethod
    def backward(ctx, dout):
        blk, kind = ctx.blk, ctx.kind
        act = blk.act_name
        k, stride = blk.kernel_size, blk.stride
        s, e_pre, e, d_pre, d, p, res, scale, mean, wt2, *sv = ctx.saved_tensors
        st1, st2, st3 = ctx.stats[:3]
        dout = dout.contiguous()
        B, OH, OW, E = d.shape
        # out = act(bn3(p) + res)
        dp, dg3, db3, dres = _bn_bwd(dout, p, st3, act, res=res, want_dres=True)
        # p = conv3(d * scale)
        w1 = blk.eca.conv.weight.detach().reshape(-1).float().contiguous()
        kk = w1.numel()
        HW = OH * OW
        dmean = torch.empty((B, E), dtype=torch.float32, device=d.device)
        dw1_img = torch.empty((B, kk), dtype=torch.float32, device=d.device)
        dweca = torch.empty(kk, dtype=torch.float32, device=d.device)
        ds = _wgrad_eca(d, dp, blk.conv3.weight, scale) if ECA_WGRAD else None
        if ds is not None:
            # dW3 and sum_hw(da * d) from one GEMM over image-aligned chunks
            dW3, ds = ds
            call("jabd_eca_gate_bwd_f32", ds.data_ptr(), 1, B, HW, E, scale.data_ptr(),
                 mean.data_ptr(), w1.data_ptr(), kk, ACT["hsigmoid"], dmean.data_ptr(),
                 dw1_img.data_ptr(), dweca.data_ptr(), _st())
            da = _dgrad(dp, blk.conv3.weight, 1, 0, OH, OW)
        else:
            dW3 = _wgrad(d, dp, blk.conv3.weight, 1, 0, ascale=scale)
            da = _dgrad(dp, blk.conv3.weight, 1, 0, OH, OW)
            nblk = max(1, min(64, HW // 256))
            part = torch.empty((B, nblk, E), dtype=torch.float32, device=d.device)
            call("jabd_eca_bwd_terms_f32", da.data_ptr(), d.data_ptr(), B, HW, E,
                 scale.data_ptr(), mean.data_ptr(), w1.data_ptr(), kk, ACT["hsigmoid"],
                 part.data_ptr(), nblk, dmean.data_ptr(), dw1_img.data_ptr(), dweca.data_ptr(),
                 _st())
        # ECA gate terms; BN2's backward applies dd = da * scale + dmean
        dd_pre, dg2, db2, _ = _bn_bwd(da, d_pre, st2, act, dys=scale, dya=dmean)
        if DW_BN_FUSE:
            de_pre, dg1, db1, dW2 = _dw_bn_bwd(dd_pre, e, wt2, k, stride, e_pre, st1, act)
        else:
            de, dW2 = _dw_bwd(dd_pre, e, wt2, k, stride)
            de_pre, dg1, db1, _ = _bn_bwd(de, e_pre, st1, act)
        dW1 = _wgrad(s, de_pre, blk.conv1.weight, 1, 0)
        # skip branch -> its input gradient, then conv1's data gradient adds it
        sk = blk.skip
        skip_grads = ()
        if kind == "identity":
            ds_skip = dres
        elif kind == "concat":
            (t_pre,) = sv
            sts0 = ctx.stats[3]
            dt, dgs, dbs, _ = _bn_bwd(dres, t_pre, sts0, "none")
            dWs = _wgrad(s, dt, sk[0].weight, 1, 0)
            dbias = _chan_sum(dt) if sk[0].bias is not None else None
            ds_skip = _dgrad_1x1_res(dt, sk[0].weight, None)
            skip_grads = (dWs, dbias, dgs, dbs)
        elif kind == "dw_concat":
            u_pre, u, t_pre, wts = sv
            sts0, sts2 = ctx.stats[3], ctx.stats[4]
            dt, dg_s3, db_s3, _ = _bn_bwd(dres, t_pre, sts2, "none")
            dWs2 = _wgrad(u, dt, sk[2].weight, 1, 0)
            dbias2 = _chan_sum(dt) if sk[2].bias is not None else None
            du = _dgrad(dt, sk[2].weight, 1, 0, u.shape[1], u.shape[2])
            du_pre, dg_s1, db_s1, _ = _bn_bwd(du, u_pre, sts0, "none")
            ds_skip, dWs0 = _dw_bwd(du_pre, s, wts, 3, 2)
            skip_grads = (dWs0, dg_s1, db_s1, dWs2, dbias2, dg_s3, db_s3)
        else:
            u_pre, wts = sv
            sts0 = ctx.stats[3]
            du_pre, dg_s1, db_s1, _ = _bn_bwd(dres, u_pre, sts0, "none")
            ds_skip, dWs0 = _dw_bwd(du_pre, s, wts, 3, 2)
            skip_grads = (dWs0, dg_s1, db_s1)
        ds = _dgrad_1x1_res(de_pre, blk.conv1.weight, ds_skip)
        grads = (dW1, dg1, db1, dW2, dg2, db2, dweca.view_as(blk.eca.conv.weight), dW3, dg3,
                 db3) + skip_grads
        return (None, ds) + grads


def _block_params(blk):
    """Parameters of a Block_eca in MNv3BlockFn's gradient order."""
    ps = [blk.conv1.weight, blk.bn1.weight, blk.bn1.bias, blk.conv2.weight, blk.bn2.weight,
          blk.bn2.bias, blk.eca.conv.weight, blk.conv3.weight, blk.bn3.weight, blk.bn3.bias]
    sk = blk.skip
    if sk is None:
        return ps
    if blk.stride == 1:
        return ps + [sk[0].weight, sk[0].bias, sk[1].weight, sk[1].bias]
    if len(sk) == 4:
        return ps + [sk[0].weight, sk[1].weight, sk[1].bias, sk[2].weight, sk[2].bias,
                     sk[3].weight, sk[3].bias]
    return ps + [sk[0].weight, sk[1].weight, sk[1].bias]


def _fused_block_ok(blk, s):
    if getattr(blk, "gate_kind", "eca") != "eca" or s.shape[3] % 4:
        return False
    bns = [blk.bn1, blk.bn2, blk.bn3] + ([m for m in blk.skip if isinstance(m, torch.nn.BatchNorm2d)]
                                          if blk.skip is not None else [])
    return all(bn.weight.shape[0] % 4 == 0 and bn.momentum is not None for bn in bns)


def _mnv3_block(blk, s):
    """Training graph of Block_eca / Block / Block_eca_G (nets/mobilenetV3.py:
    :140-150, :81-91, :198-208): the gate is ECA on the project conv's load,
    SE or BECA applied explicitly, or none."""
    if FUSED_BLOCKS and _fused_block_ok(blk, s):
        ps = _block_params(blk)
        # a parameter that is None (no conv bias) is passed as None
        return MNv3BlockFn.apply(blk, s, *ps)
    act = blk.act_name
    e = bn_act(conv(s, blk.conv1), blk.bn1, act)
    d = bn_act(DwConvFn.apply(e, blk.conv2.weight, blk.stride), blk.bn2, act)
    gate = getattr(blk, "gate_kind", "eca")
    if gate == "eca":
        p = EcaConvFn.apply(d, blk.eca.conv.weight, blk.conv3.weight, 1, 0, "hsigmoid")
    else:
        if gate == "se":
            from .modules import ScaleFn, se_scale_train
            d = ScaleFn.apply(d, se_scale_train(blk.se, d))
        elif gate == "beca":
            from .ops import BecaFn
            d = BecaFn.apply(d, blk.eca.conv.weight.reshape(-1))
        p = conv(d, blk.conv3)
    sk = blk.skip
    if sk is None:
        res = s
    elif blk.stride == 1:
        res = bn_act(conv(s, sk[0]), sk[1])
    elif len(sk) == 4:
        t = bn_act(DwConvFn.apply(s, sk[0].weight, 2), sk[1])
        res = bn_act(conv(t, sk[2]), sk[3])
    else:
        res = bn_act(DwConvFn.apply(s, sk[0].weight, 2), sk[1])
    return bn_act(p, blk.bn3, act, res=res)


class R50BlockFn(torch.autograd.Function):
    """One torchvision Bottleneck (nets/resnet_pytorch_r.py:122-143) forward
    and backward as a single autograd node, so the gradient reaching the
    block input from its two consumers (conv1 and the identity / downsample
    branch) is summed in the epilogue of conv1's data-gradient GEMM instead
    of by an autograd add over the block input (an ATen elementwise kernel
    per block, ~15 ms per C3 step).  Inputs: the block, x, then the
    parameters in _r50_params order."""

    @staticmethod
    def forward(ctx, blk, prev, info, x, *params):
        """prev: the link record of the bottleneck whose output x is (None:
        x came from elsewhere); info: this block's record, filled here."""
        stride = blk.stride
        B, H, W, _ = x.shape
        # each conv's GEMM epilogue also takes its BatchNorm's batch statistics
        t1p, bs1 = _conv_fwd_stats(x, blk.conv1.weight, blk.bn1)
        t1, st1 = _bn_fwd(t1p, blk.bn1, "relu", stats=bs1)
        t2p, bs2 = _conv_fwd_stats(t1, blk.conv2.weight, blk.bn2, stride, 1)
        t2, st2 = _bn_fwd(t2p, blk.bn2, "relu", stats=bs2)
        t3p, bs3 = _conv_fwd_stats(t2, blk.conv3.weight, blk.bn3)
        ds = blk.downsample
        saved = ()
        if ds is not None:
            ip, bss = _conv_fwd_stats(x, ds[0].weight, ds[1], stride, 0)
            idn, sts = _bn_fwd(ip, ds[1], "none", stats=bss)
            saved = (ip,)
            ctx.sts = sts
        else:
            idn = x
        out, st3 = _bn_fwd(t3p, blk.bn3, "relu", res=idn, stats=bs3)
        ctx.blk, ctx.st = blk, (st1, st2, st3)
        ctx.hw = (H, W)
        ctx.prev, ctx.info = prev, info
        if info is not None:
            # what the next bottleneck's conv1 data gradient needs to hand this
            # block dz and bn3's sums instead of dout (R50_BN3_LINK)
            info.update(x3=t3p, st3=st3, rows=None, dz=None)
        ctx.save_for_backward(x, t1p, t1, t2p, t2, t3p, idn, *saved)
        return out

    @staticmethod
    def backward(ctx, dout):
        blk = ctx.blk
        stride = blk.stride
        H, W = ctx.hw
        x, t1p, t1, t2p, t2, t3p, idn, *sv = ctx.saved_tensors
        st1, st2, st3 = ctx.st
        dout = dout.contiguous()
        info = ctx.info
        if info is not None and info["rows"] is not None and info["dz"] == dout.data_ptr():
            # the next block's conv1 data gradient already wrote dz = dout *
            # [out > 0] and bn3's sums: only the apply pass is left, and dz
            # is the identity branch's gradient
            dp3, dg3, db3, _ = _bn_bwd_rows(dout, t3p, st3, "none", info["rows"])
            dres = dout
        else:
            dp3, dg3, db3, dres = _bn_bwd(dout, t3p, st3, "relu", res=idn, want_dres=True)
        if info is not None:
            info.clear()
        dW3 = _wgrad(t2, dp3, blk.conv3.weight, 1, 0)
        # the data-gradient GEMMs also take the next BatchNorm backward's sums
        dt2, pt2 = _dgrad_bn_sums(dp3, blk.conv3.weight, 1, 0, t2.shape[1], t2.shape[2], t2p,
                                  st2, "relu")
        dp2, dg2, db2, _ = (_bn_bwd_rows(dt2, t2p, st2, "relu", pt2) if pt2 is not None
                            else _bn_bwd(dt2, t2p, st2, "relu"))
        dW2 = _wgrad(t1, dp2, blk.conv2.weight, stride, 1)
        dt1, pt1 = _dgrad_bn_sums(dp2, blk.conv2.weight, stride, 1, H, W, t1p, st1, "relu")
        dp1, dg1, db1, _ = (_bn_bwd_rows(dt1, t1p, st1, "relu", pt1) if pt1 is not None
                            else _bn_bwd(dt1, t1p, st1, "relu"))
        dW1 = _wgrad(x, dp1, blk.conv1.weight, 1, 0)
        grads = (dW1, dg1, db1, dW2, dg2, db2, dW3, dg3, db3)
        if blk.downsample is not None:
            (ip,) = sv
            ds = blk.downsample
            dip, dgs, dbs, _ = _bn_bwd(dres, ip, ctx.sts, "none")
            dWs = _wgrad(x, dip, ds[0].weight, stride, 0)
            ds_skip = _dgrad(dip, ds[0].weight, stride, 0, H, W)
            grads += (dWs, dgs, dbs)
        else:
            ds_skip = dres
        prev = ctx.prev
        if prev is not None and prev.get("x3") is not None:
            dx, rows = _dgrad_1x1_res_bn3(dp1, blk.conv1.weight, ds_skip, x, prev["x3"],
                                          prev["st3"])
            prev["rows"], prev["dz"] = rows, (dx.data_ptr() if rows is not None else None)
        else:
            dx = _dgrad_1x1_res(dp1, blk.conv1.weight, ds_skip)
        return (None, None, None, dx) + grads


def _r50_params(blk):
    ps = [blk.conv1.weight, blk.bn1.weight, blk.bn1.bias, blk.conv2.weight, blk.bn2.weight,
          blk.bn2.bias, blk.conv3.weight, blk.bn3.weight, blk.bn3.bias]
    if blk.downsample is not None:
        ps += [blk.downsample[0].weight, blk.downsample[1].weight, blk.downsample[1].bias]
    return ps


def _r50_fused_ok(blk, x):
    convs = [blk.conv1, blk.conv2, blk.conv3] + ([blk.downsample[0]] if blk.downsample is not None
                                                 else [])
    bns = [blk.bn1, blk.bn2, blk.bn3] + ([blk.downsample[1]] if blk.downsample is not None
                                         else [])
    return (R50_FUSED and x.shape[3] % 4 == 0 and blk.conv1.kernel_size == (1, 1) and
            blk.conv1.stride == (1, 1) and all(c.bias is None for c in convs) and
            all(b.weight.shape[0] % 4 == 0 and b.momentum is not None for b in bns))


# JABD_R50_FUSED=0: the bottleneck as per-op autograd nodes (A/B)
R50_FUSED = __import__("os").environ.get("JABD_R50_FUSED", "1") != "0"
# JABD_R50_BN3_LINK=0: every bottleneck takes its bn3 backward from dout
# (jabd_bn_act_bwd_ex_f32's two passes) instead of from the dz + sums the
# next bottleneck's conv1 data gradient writes (A/B)
R50_BN3_LINK = __import__("os").environ.get("JABD_R50_BN3_LINK", "1") != "0"


def _r50_block(blk, x):
    if _r50_fused_ok(blk, x):
        x = x.contiguous()
        # link to the producing bottleneck when x IS its output object (its
        # only consumer is this block: the _train_forward chain; a fork or
        # any other use gives a different object)
        rec = getattr(x, "_jabd_r50_link", None) if R50_BN3_LINK else None
        prev = rec[1] if rec is not None and rec[0]() is x else None
        info = {} if R50_BN3_LINK else None
        out = R50BlockFn.apply(blk, prev, info, x, *_r50_params(blk))
        if info is not None:
            out._jabd_r50_link = (weakref.ref(out), info)
        return out
    t = bn_act(conv(x, blk.conv1), blk.bn1, "relu")
    t = bn_act(conv(t, blk.conv2, blk.stride, 1), blk.bn2, "relu")
    t = conv(t, blk.conv3)
    if blk.downsample is not None:
        idn = bn_act(conv(x, blk.downsample[0], blk.stride), blk.downsample[1])
    else:
        idn = x
    return bn_act(t, blk.bn3, "relu", res=idn)


def _nlm_params(nlm):
    return (nlm.f_query.weight, nlm.f_query.bias, nlm.f_key.weight, nlm.f_key.bias,
            nlm.f_value.weight, nlm.f_value.bias, nlm.W.weight, nlm.W.bias)


def nlm_train(nlm, src, lateral=None, nw=None):
    """ch=4: lateral + NLM(nearest(src)) fused (lateral=None: NLM(src)).
    Other widths: lateral + NLM(src) composed from ConvFn / AdaptivePoolFn /
    NlmAttnFn (src already at the output size).  nw: the module's eight
    parameters or autograd aliases of them (the FPN runs one NLM twice)."""
    nw = _nlm_params(nlm) if nw is None else nw
    if nlm.ch == 4:
        return NlmFn.apply(src, lateral, *nw, tuple(nlm.psp.sizes))
    from .modules import AdaptivePoolFn
    x = src.contiguous()
    B, h, w, C = x.shape
    sizes = tuple(nlm.psp.sizes)
    S = sum(s_ * s_ for s_ in sizes)
    q = ConvFn.apply(x, nw[0], nw[1], 1, 0, False)
    pooled = AdaptivePoolFn.apply(x, sizes).view(B, S, 1, C)
    kp = ConvFn.apply(pooled, nw[2], nw[3], 1, 0, False).view(B, S, nlm.ch)
    vp = ConvFn.apply(pooled, nw[4], nw[5], 1, 0, False).view(B, S, nlm.ch)
    y = ConvFn.apply(NlmAttnFn.apply(q, kp, vp), nw[6], nw[7], 1, 0, False)
    return Add3Fn.apply(y, x, lateral)


def fpn_up_train(fpn, nlm, src, lateral, nw=None):
    """lateral + [NLM](up(src -> lateral's size)) in training mode; nw: the
    NLM's parameters (or aliases, see nlm_train)."""
    mode = getattr(fpn, "upsample_mode", "nearest")
    if nlm is None:
        if mode == "nearest":
            return UpAddFn.apply(src, lateral)
        return Add3Fn.apply(UpsampleFn.apply(src, lateral.shape[1], lateral.shape[2], mode),
                            lateral, None)
    if mode == "nearest" and nlm.ch == 4:
        return nlm_train(nlm, src, lateral, nw)
    up = UpsampleFn.apply(src, lateral.shape[1], lateral.shape[2], mode)
    if nlm.ch == 4:
        return Add3Fn.apply(nlm_train(nlm, up, None, nw), lateral, None)
    return nlm_train(nlm, up, lateral, nw)


def fpn_train(fpn, feats, nlm=None, eca_ws=None, gate="sigmoid"):
    """FPN forward (nets/retinaface_r.py:169-207; nlm=None: nets/layers.py:83-119;
    bicubic: train_mobilenetV3_ecagai.py:254-285) in training mode; eca_ws:
    the three input ECA Conv1d weights — mean-pool ECA applied on the lateral
    convs' operand load (nets/retinaface_r.py:313-315), or with gate="beca"
    the std-pool BECA (train_mobilenetV3_ecagai.py:415-418)."""
    lk = fpn.leaky
    outs = (fpn.output1, fpn.output2, fpn.output3)
    lat = []
    for i, (f, o) in enumerate(zip(feats, outs)):
        if eca_ws is not None and gate == "beca":
            from .ops import BecaFn
            y = conv(BecaFn.apply(f, eca_ws[i].reshape(-1)), o[0])
        elif eca_ws is not None:
            y = EcaConvFn.apply(f, eca_ws[i], o[0].weight, 1, 0, "sigmoid")
        else:
            y = conv(f, o[0])
        lat.append(bn_act(y, o[1], "leaky", lk))
    o1, o2, o3 = lat

    # one NLM module serves both up-merges: its parameters get one alias per
    # use, so their two gradients are summed by ForkFn, not by autograd
    nws = [None, None]
    if nlm is not None:
        nws = list(zip(*[fork(p_, 2) for p_ in _nlm_params(nlm)]))

    def up(s_, l_):
        return fpn_up_train(fpn, nlm, s_, l_, nws.pop(0))
    o3, o3u = fork(o3, 2)  # to the SSH and up-sampled into o2
    o2 = bn_act(conv(up(o3u, o2), fpn.merge2[0], 1, 1), fpn.merge2[1], "leaky", lk)
    o2, o2u = fork(o2, 2)
    o1 = bn_act(conv(up(o2u, o1), fpn.merge1[0], 1, 1), fpn.merge1[1], "leaky", lk)
    return [o1, o2, o3]


def ssh_train(ssh, o, eca_w=None, padded_out=False):
    """SSH forward (nets/layers.py:56-68) in training mode; eca_w: the head's
    eca_fpn Conv1d weight (or two autograd aliases of it, one per use)
    applied on the two input convs' operand load.
    padded_out: when the quarter branches are zero-padded to a multiple of 4
    channels, return (padded tensor, (half, q, qp) layout) instead of copying
    the real channels out (the heads read the padded layout)."""
    q = ssh.conv5X5_1[0].out_channels
    qp = _pad_to4(q)
    # o feeds two convs, and so does the eca weight (one alias each, ForkFn)
    ins = list(zip(fork(o, 2), fork(eca_w, 2) if isinstance(eca_w, torch.Tensor) else
                   (eca_w if eca_w is not None else (None, None))))

    def first(w):
        oi, ei = ins.pop(0)
        if ei is not None:
            return EcaConvFn.apply(oi, ei, w, 1, 1, "sigmoid")
        return ConvFn.apply(oi, w, None, 1, 1, False)

    a = first(ssh.conv3X3[0].weight)
    bns = (ssh.conv3X3[1], ssh.conv5X5_2[1], ssh.conv7x7_3[1])
    if qp == q:
        b1 = bn_act(first(ssh.conv5X5_1[0].weight), ssh.conv5X5_1[1], "leaky", ssh.leaky)
        b1a, b1b = fork(b1, 2)
        b = ConvFn.apply(b1a, ssh.conv5X5_2[0].weight, None, 1, 1, False)
        c1 = bn_act(ConvFn.apply(b1b, ssh.conv7X7_2[0].weight, None, 1, 1, False),
                    ssh.conv7X7_2[1], "leaky", ssh.leaky)
        c = ConvFn.apply(c1, ssh.conv7x7_3[0].weight, None, 1, 1, False)
        gb, stats = [], []
        for bn in bns:
            gb += [bn.weight, bn.bias]
            stats.append((bn.running_mean, bn.running_var, bn.momentum, bn.eps))
            _count_batch(bn)
        f = SshTailFn.apply(a, b, c, *gb, stats)
        return (f, None) if padded_out else f
    # 10-channel quarter branches stored as qp channels: every padded weight,
    # BN parameter and running statistic in one PadFn launch, the running
    # statistics cropped back in one launch after the forward
    convs = (ssh.conv5X5_1[0], ssh.conv5X5_2[0], ssh.conv7X7_2[0], ssh.conv7x7_3[0])
    pbns = (ssh.conv5X5_1[1], ssh.conv7X7_2[1], ssh.conv5X5_2[1], ssh.conv7x7_3[1])
    spec = [(convs[0].weight, (qp,) + tuple(convs[0].weight.shape[1:]), 0.0)]
    spec += [(cv.weight, (qp, qp) + tuple(cv.weight.shape[2:]), 0.0) for cv in convs[1:]]
    for bn in pbns:
        spec += [(bn.weight, (qp,), 0.0), (bn.bias, (qp,), 0.0),
                 (bn.running_mean, (qp,), 0.0), (bn.running_var, (qp,), 1.0)]
    pt = _padded(spec)
    w51, w52, w72, w73 = pt[:4]
    pb = [pt[4 + 4 * i:8 + 4 * i] for i in range(4)]  # (g, b, rm, rv) per padded BN

    def bn_p(x, i):
        g, bt, rm, rv = pb[i]
        y = BnActFn.apply(x, g, bt, None, rm, rv, "leaky", ssh.leaky, pbns[i].momentum,
                          pbns[i].eps)
        _count_batch(pbns[i])
        return y

    b1a, b1b = fork(bn_p(first(w51), 0), 2)
    b = ConvFn.apply(b1a, w52, None, 1, 1, False)
    c1 = bn_p(ConvFn.apply(b1b, w72, None, 1, 1, False), 1)
    c = ConvFn.apply(c1, w73, None, 1, 1, False)
    bn0 = bns[0]
    gb = [bn0.weight, bn0.bias, pb[2][0], pb[2][1], pb[3][0], pb[3][1]]
    stats = [(bn0.running_mean, bn0.running_var, bn0.momentum, bn0.eps),
             (pb[2][2], pb[2][3], pbns[2].momentum, pbns[2].eps),
             (pb[3][2], pb[3][3], pbns[3].momentum, pbns[3].eps)]
    for bn in bns:
        _count_batch(bn)
    f = SshTailFn.apply(a, b, c, *gb, stats)
    with torch.no_grad():
        F.window_copies([(pb[i][2 + j], (bn.running_mean, bn.running_var)[j], 0.0)
                         for i, bn in enumerate(pbns) for j in (0, 1)])
    half = a.shape[3]
    if padded_out:
        return f, (half, q, qp)
    # drop the zero pad channels of the 10-channel branches
    f = torch.cat([f[..., :half], f[..., half:half + q], f[..., half + qp:half + qp + q]], -1)
    return f.contiguous()


def _head(m, feats, eca_names, nlm):
    gate = getattr(m, "head_gate", "sigmoid")
    o1, o2, o3 = fpn_train(m.fpn, feats, nlm,
                           [getattr(m, n).conv.weight for n in eca_names], gate)
    ew = m.eca_fpn.conv.weight
    if gate == "beca":
        from .ops import BecaFn
        outs = [ssh_train(ssh, BecaFn.apply(o, e.reshape(-1)), padded_out=True)
                for o, ssh, e in zip((o1, o2, o3), (m.ssh1, m.ssh2, m.ssh3), fork(ew, 3))]
    else:  # the shared eca weight: one alias per use (two per SSH)
        ews = fork(ew, 6)
        outs = [ssh_train(ssh, o, ews[2 * i:2 * i + 2], padded_out=True)
                for i, (o, ssh) in enumerate(zip((o1, o2, o3), (m.ssh1, m.ssh2, m.ssh3)))]
    wb = []
    for i in range(3):
        for h in (m.BboxHead[i], m.ClassHead[i], m.LandmarkHead[i]):
            wb += [h.conv1x1.weight, h.conv1x1.bias]
    return HeadsFn.apply(*[f for f, _ in outs], tuple(ci for _, ci in outs), *wb)


def train_forward(model, kind, x):
    if model.mode != "train":
        raise NotImplementedError("training-mode forward returns logits (mode='train'); the "
                                  "reference's training scripts construct RetinaFace that way")
    with _BatchCounts():
        return _train_forward(model, kind, x.contiguous())


def _train_forward(model, kind, x):
    if kind == "mnv3":
        body = model.body
        s = bn_act(conv(x, body.conv1, 2, 1, nchw_in=True), body.bn1, "hswish")
        feats = []
        from .engine import mnv3_stages
        stages = list(mnv3_stages(body))
        for i, stage in enumerate(stages):
            for blk in stage:
                s = _mnv3_block(blk, s)
            if i + 1 < len(stages):  # feeds the next stage and the FPN
                s, f = fork(s, 2)
            else:
                f = s
            feats.append(f)
        return _head(model, feats, getattr(model, "eca_names", ("eca_40", "eca_80", "eca_160")),
                     model.fpn.nlm)
    body = model.body
    s = bn_act(conv(x, body.conv1, 2, 3, nchw_in=True), body.bn1, "relu")
    s = MaxPoolFn.apply(s)
    feats = []
    for i in (1, 2, 3, 4):
        for blk in getattr(body, f"layer{i}"):
            s = _r50_block(blk, s)
        if i in (2, 3):  # feeds the next stage and the FPN
            s, f = fork(s, 2)
            feats.append(f)
        elif i == 4:
            feats.append(s)
    return _head(model, feats, ("eca_64", "eca_128", "eca_256"), model.fpn.Nlm)
