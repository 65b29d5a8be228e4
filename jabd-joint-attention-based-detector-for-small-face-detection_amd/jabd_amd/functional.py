"""NHWC fp32 layer primitives over libjabd (conv, depthwise, ECA, NLM, heads).

Activations are torch tensors [B, H, W, C] (a channel slice of a wider
tensor is described by (tensor, c0)).  Weights arrive pre-folded and
pre-packed (see `pack_conv`); every call launches on torch's current stream
and returns without synchronising.
"""
import ctypes
import threading

import torch

from ._lib import ConvArgs, DwArgs, ExpDwArgs, call, lib

ACT = {"none": 0, "relu": 1, "leaky": 2, "hswish": 3, "hsigmoid": 4, "sigmoid": 5}

# Test hook (tests/_kinks.py), None in use: when set, the training forward
# hands it the operands from which each backward kernel derives the region
# of a piecewise activation (ReLU / LeakyReLU / Hardswish / Hardsigmoid) or a
# max-pool argmax, so the float64 oracle can be run with this path's own
# masks.  tap(kind, *operands); kinds: "bn", "eca", "beca", "act", "ssh",
# "maxpool", and "stats" (src, x, mean, invstd, eps: every BatchNorm's batch
# statistics with the tensor they were taken of and the kernel that took
# them, for the at-size statistics checks).
KINK_TAP = None

# Split-K for small-grid k x k convs (conv32.hip m32_ksplit).  It regroups
# the fp32 K sum, so an image's outputs then depend (in rounding only) on the
# batch it was run in.  Off by default (batched eval is batch-invariant: an
# image gives the same bits at any batch size); the bs1 predict path turns it
# on for its forward (jabd_amd.predict, `with split_k():`), where the R50's
# late 3x3 convs would otherwise fill a few dozen workgroups.  The setting is
# per thread, so a threaded server running bs1 predict beside batched eval
# cannot flip the other thread's form.
_KSPLIT = threading.local()


def ksplit_enabled():
    return getattr(_KSPLIT, "on", False)


class split_k:
    """Context manager: split-K on (or off) for the convs this thread launches
    inside it."""

    def __init__(self, enabled=True):
        self.enabled = enabled

    def __enter__(self):
        self.prev = ksplit_enabled()
        _KSPLIT.on = self.enabled
        return self

    def __exit__(self, *exc):
        _KSPLIT.on = self.prev


def tap(kind, *operands):
    if KINK_TAP is not None:
        KINK_TAP(kind, *operands)


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t):
    return t.data_ptr() if t is not None else None


def _check(name, t):
    if not t.is_cuda or t.dtype != torch.float32:
        raise RuntimeError(f"{name}: needs a float32 GPU tensor (no CPU fallback), got "
                           f"{t.dtype} on {t.device}")


# ----------------------------------------------------------------------------- packing
class PackedConv:
    """Weights of one implicit-GEMM conv in the MFMA fragment order.

    w2d: [K, Cout] with k = (kh*KW + kw)*Cin + ci (+ K-concatenated rows).
    Stored as float4 [Kc][Ntiles][64 lanes], lane = 16*g + j holding
    W[16kc + 4g + e][16nt + j] for e = 0..3 (conv.hip header).
    """

    def __init__(self, w2d, bias, KH, KW, Cin, Cin2=0):
        K, cout = w2d.shape
        self.KH, self.KW, self.Cin, self.Cin2, self.Cout = KH, KW, Cin, Cin2, cout
        self.tn = int(lib().jabd_conv_pack_tn(cout))
        tiles = (cout + 15) // 16
        self.Ntiles = (tiles + self.tn - 1) // self.tn * self.tn
        self.Kc = (K + 15) // 16
        wp = torch.zeros((self.Kc * 16, self.Ntiles * 16), dtype=torch.float32, device=w2d.device)
        wp[:K, :cout] = w2d
        # [Kc, g, e, Ntiles, j] -> [Kc, Ntiles, g, j, e]
        wp = wp.view(self.Kc, 4, 4, self.Ntiles, 16).permute(0, 3, 1, 4, 2).contiguous()
        self.w = wp
        self.bias = bias.contiguous().float() if bias is not None else None
        self.w32 = None
        if (KH == 1 and KW == 1) or (Cin % 32 == 0 and not Cin2):
            self._pack32(w2d)

    def _pack32(self, w2d):
        """Second packing for the 32x32x2 1x1 kernel (csrc/conv32.hip):
        float4 [K8][ntiles32][64 lanes], lane = 32h + j holding
        W[8k8 + 4h + e][32nt + j] for e = 0..3; K padded to 32."""
        K, cout = w2d.shape
        self.tn32 = int(lib().jabd_conv_pack_tn32(cout))
        nt = (cout + 31) // 32
        self.ntiles32 = (nt + self.tn32 - 1) // self.tn32 * self.tn32
        k8 = (K + 31) // 32 * 4
        wp = torch.zeros((k8 * 8, self.ntiles32 * 32), dtype=torch.float32, device=w2d.device)
        wp[:K, :cout] = w2d
        # [K8, h, e, NT, j] -> [K8, NT, h, j, e]
        self.w32 = wp.view(k8, 2, 4, self.ntiles32, 32).permute(0, 3, 1, 4, 2).contiguous()


def pack_weight_device(weight, transposed=False):
    """PackedConv of a raw torch conv weight [Cout, Cin, KH, KW] built by one
    device kernel (jabd_conv_pack_f32) — the same layouts as PackedConv(
    conv_weight_2d(w), ...) without the host-side zeros / copies / permutes.
    transposed: the data-gradient form (input and output channels swapped)."""
    w = weight.detach()
    if w.dtype != torch.float32 or not w.is_contiguous():
        w = w.float().contiguous()
    cout, cin, kh, kw = w.shape
    pcin, pcout = (cout, cin) if transposed else (cin, cout)
    pk = PackedConv.__new__(PackedConv)
    pk.KH, pk.KW, pk.Cin, pk.Cin2, pk.Cout = kh, kw, pcin, 0, pcout
    pk.tn = int(lib().jabd_conv_pack_tn(pcout))
    tiles = (pcout + 15) // 16
    pk.Ntiles = (tiles + pk.tn - 1) // pk.tn * pk.tn
    K = kh * kw * pcin
    pk.Kc = (K + 15) // 16
    pk.bias = None
    pk.w = torch.empty((pk.Kc, pk.Ntiles, 4, 16, 4), dtype=torch.float32, device=w.device)
    pk.w32 = None
    k8 = nt32 = 0
    if (kh == 1 and kw == 1) or pcin % 32 == 0:
        pk.tn32 = int(lib().jabd_conv_pack_tn32(pcout))
        nt = (pcout + 31) // 32
        pk.ntiles32 = (nt + pk.tn32 - 1) // pk.tn32 * pk.tn32
        k8 = (K + 31) // 32 * 4
        nt32 = pk.ntiles32
        pk.w32 = torch.empty((k8, nt32, 2, 32, 4), dtype=torch.float32, device=w.device)
    call("jabd_conv_pack_f32", w.data_ptr(), cout, cin, kh, kw, 1 if transposed else 0, pk.Kc,
         pk.Ntiles, pk.w.data_ptr(), k8, nt32, _ptr(pk.w32), _stream())
    return pk


def conv_weight_2d(weight):
    """nn.Conv2d weight [Cout, Cin, KH, KW] -> [KH*KW*Cin, Cout] (tap-major)."""
    cout, cin, kh, kw = weight.shape
    return weight.permute(2, 3, 1, 0).reshape(kh * kw * cin, cout)


def bn_fold(bn, conv_bias=None):
    """Eval BatchNorm2d as (scale, shift) per channel; conv bias folded in."""
    s = bn.weight / torch.sqrt(bn.running_var + bn.eps)
    t = bn.bias - bn.running_mean * s
    if conv_bias is not None:
        t = t + conv_bias * s
    return s, t


def pack_conv(conv, bn=None, extra=None, cin_pad=None, cout_pad=None):
    """Fold (conv [+ bn]) [+ extra K-concatenated (w2d, shift)] into PackedConv.

    cin_pad / cout_pad zero-extend the input / output channels (a 10-channel
    SSH tensor stored as 12 channels takes the 16-byte vector path; the extra
    output channels compute exactly 0)."""
    w2d, bias, kh, kw, cin, cin2 = _fold_conv(conv, bn, extra, cin_pad, cout_pad)
    return PackedConv(w2d, bias, kh, kw, cin, cin2)


def pack_conv_cat(parts, cin_pad=None):
    """Two or more convolutions of the same input fused along N (output
    channels concatenated in order): parts = [(conv, bn, cout_pad), ...].
    Used with conv(..., y2=, nsplit=) to write the parts to separate tensors."""
    ws, bs = [], []
    for conv, bn, cout_pad in parts:
        w2d, bias, kh, kw, cin, _ = _fold_conv(conv, bn, None, cin_pad, cout_pad)
        ws.append(w2d)
        bs.append(bias if bias is not None else w2d.new_zeros(w2d.shape[1]))
    return PackedConv(torch.cat(ws, 1).contiguous(), torch.cat(bs).contiguous(), kh, kw, cin)


def _fold_conv(conv, bn, extra, cin_pad, cout_pad):
    wt = conv.weight.detach().float()
    cb = conv.bias.detach().float() if conv.bias is not None else None
    if bn is not None:
        s, t = bn_fold(bn, cb)
        wt = wt * s[:, None, None, None]
        bias = t
    else:
        bias = cb
    cout, cin = wt.shape[0], wt.shape[1]
    if cin_pad is not None and cin_pad > cin:
        wt = torch.cat([wt, wt.new_zeros((cout, cin_pad - cin) + tuple(wt.shape[2:]))], 1)
        cin = cin_pad
    if cout_pad is not None and cout_pad > cout:
        wt = torch.cat([wt, wt.new_zeros((cout_pad - cout,) + tuple(wt.shape[1:]))], 0)
        bias = torch.cat([bias if bias is not None else wt.new_zeros(cout),
                          wt.new_zeros(cout_pad - cout)])
    w2d = conv_weight_2d(wt)
    cin2 = 0
    if extra is not None:
        w2, t2 = extra
        cin2 = w2.shape[0]
        w2d = torch.cat([w2d, w2], 0)
        bias = t2 if bias is None else bias + t2
    kh, kw = conv.weight.shape[2], conv.weight.shape[3]
    return (w2d.detach(), bias.detach() if bias is not None else None, kh, kw, cin, cin2)


def pack_dw(conv, bn):
    """Depthwise conv + BN -> (w [k*k][C] tap-major, bias [C])."""
    c, _, k, _ = conv.weight.shape
    s, t = bn_fold(bn, conv.bias.detach().float() if conv.bias is not None else None)
    w = (conv.weight.detach().float().view(c, k * k) * s[:, None]).t().contiguous()
    return w, t.detach().contiguous()


# ----------------------------------------------------------------------------- kernels
_CONV_DBG = 0  # load/store skip mask for tools/convbench.py timing experiments only


def conv(x, pk, stride=1, pad=0, act="none", slope=0.0, ascale=None, x2=None, x2_stride=1,
         res=None, out=None, out_c0=0, nchw_in=False, x_c0=0, y2=None, y2_c0=0, nsplit=0,
         act2="none", slope2=0.0):
    """Implicit-GEMM conv.  x [B,H,W,C*] NHWC (or NCHW input if nchw_in).

    Split output: with y2 [B,OH,OW,C2], output channels >= nsplit go to y2 at
    channel y2_c0 + (n - nsplit) with act2 / slope2."""
    _check("conv.x", x)
    if nchw_in:
        B, cin, H, W = x.shape
        x_bs, x_ps = cin * H * W, 1
    else:
        B, H, W, ctot = x.shape
        x_bs, x_ps = H * W * ctot, ctot
    OH = (H + 2 * pad - pk.KH) // stride + 1
    OW = (W + 2 * pad - pk.KW) // stride + 1
    if out is None:
        out = torch.empty((B, OH, OW, pk.Cout), dtype=torch.float32, device=x.device)
        out_c0 = 0
    a = ConvArgs()
    a.x, a.x_bs, a.x_ps, a.x_c0 = x.data_ptr(), x_bs, x_ps, x_c0
    a.B, a.H, a.W, a.Cin = B, H, W, pk.Cin
    if x2 is not None:
        a.x2, a.x2_bs, a.x2_ps, a.Cin2 = x2.data_ptr(), x2.stride(0), x2.shape[3], pk.Cin2
        a.x2_W, a.x2_stride = x2.shape[2], x2_stride
    if ascale is not None:
        a.ascale, a.ascale_bs = ascale.data_ptr(), ascale.shape[1]
    a.w = pk.w.data_ptr()
    a.bias = _ptr(pk.bias)
    if res is not None:
        a.res, a.res_bs, a.res_ps, a.res_c0 = res.data_ptr(), res.stride(0), res.shape[3], 0
    a.y, a.y_bs, a.y_ps, a.y_c0 = out.data_ptr(), out.stride(0), out.shape[3], out_c0
    a.OH, a.OW, a.Cout, a.Ntiles, a.tn, a.Kc = OH, OW, pk.Cout, pk.Ntiles, pk.tn, pk.Kc
    if pk.w32 is not None and not nchw_in:
        a.w32, a.ntiles32, a.tn32 = pk.w32.data_ptr(), pk.ntiles32, pk.tn32
    a.KH, a.KW, a.stride, a.pad = pk.KH, pk.KW, stride, pad
    a.act, a.slope = ACT[act], float(slope)
    a.nchw_in = 1 if nchw_in else 0
    a.reserved1 = _CONV_DBG
    ws = None
    if ksplit_enabled() and pk.w32 is not None and not nchw_in and y2 is None:
        # a conv on the 32x32 kernel whose output grid cannot fill the device
        # (bs1) may split its K reduction over workgroups: give it the
        # workspace it asks for
        nbytes = int(lib().jabd_conv_workspace_size(ctypes.byref(a)))
        if nbytes > 0:
            ws = torch.empty(nbytes // 4, dtype=torch.float32, device=x.device)
            a.ws, a.ws_bytes = ws.data_ptr(), nbytes
    if y2 is not None:
        _check("conv.y2", y2)
        a.y2, a.y2_bs, a.y2_ps, a.y2_c0 = y2.data_ptr(), y2.stride(0), y2.shape[3], y2_c0
        a.nsplit, a.act2, a.slope2 = nsplit, ACT[act2], float(slope2)
    call("jabd_conv2d_nhwc_f32", ctypes.byref(a), _stream())
    return out


def stem(x, w, bias, act):
    """MobileNetV3 stem: NCHW [B,3,H,W] -> NHWC [B,H/2,W/2,16] (w [27][16])."""
    _check("stem.x", x)
    B, _, H, W = x.shape
    OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    y = torch.empty((B, OH, OW, 16), dtype=torch.float32, device=x.device)
    call("jabd_stem_nchw_f32", x.data_ptr(), B, H, W, w.data_ptr(), bias.data_ptr(), ACT[act],
         y.data_ptr(), _stream())
    return y


def dw_nblk(B, OH, OW, C):
    return int(lib().jabd_dw_nblk(B, OH, OW, C))


def dwconv(x, w, bias, k, stride, act="none", slope=0.0, partials=False):
    """Depthwise k x k conv (pad k//2) + folded BN + act; optional ECA partial sums."""
    _check("dw.x", x)
    B, H, W, C = x.shape
    pad = k // 2
    OH = (H + 2 * pad - k) // stride + 1
    OW = (W + 2 * pad - k) // stride + 1
    y = torch.empty((B, OH, OW, C), dtype=torch.float32, device=x.device)
    part = None
    a = DwArgs()
    a.x, a.x_bs, a.x_ps = x.data_ptr(), x.stride(0), C
    a.B, a.H, a.W, a.C = B, H, W, C
    a.w, a.bias = w.data_ptr(), _ptr(bias)
    a.y, a.y_bs, a.y_ps = y.data_ptr(), y.stride(0), C
    a.OH, a.OW, a.k, a.stride, a.pad, a.act = OH, OW, k, stride, pad, ACT[act]
    a.slope = float(slope)
    if partials:
        nb = dw_nblk(B, OH, OW, C)
        part = torch.empty((B, nb, C), dtype=torch.float32, device=x.device)
        a.nblk, a.part = nb, part.data_ptr()
    call("jabd_dwconv_nhwc_f32", ctypes.byref(a), _stream())
    return y, part


_XD_DBG = 0  # kernel-phase skip mask for tools/convbench.py timing experiments only


def expand_dw(x, pk, w, bias, k, stride, act="none", partials=True, skip=None, pre=None):
    """Fused expand 1x1 (PackedConv pk, folded BN) + act -> depthwise k x k
    (pad k//2, folded BN) + act; returns (y, ECA partials [B, nblk, E]).
    skip = (w [9][Cin], bias [Cin]) (stride 2): the block's dw3x3/s2 skip
    branch computed from the same input tile; returns (y, partials, t).
    pre = (pk_prev, gate [B, Cin], res, act_prev): x is the previous block's
    depthwise output and that block's project act_prev(pk_prev(gate * x) +
    res) runs inside the kernel in front of the expand (the 3x3/s2 Cin-16
    skip form; jabd_expdw_args.pw)."""
    _check("expand_dw.x", x)
    B, H, W, C = x.shape
    if pk.KH != 1 or pk.KW != 1 or pk.Cin != C or pk.Cin2:
        raise ValueError("expand_dw: pk must be a plain 1x1 conv over all input channels")
    E = pk.Cout
    pad = k // 2
    OH = (H + 2 * pad - k) // stride + 1
    OW = (W + 2 * pad - k) // stride + 1
    y = torch.empty((B, OH, OW, E), dtype=torch.float32, device=x.device)
    a = ExpDwArgs()
    a.x, a.x_bs, a.x_ps, a.Cin = x.data_ptr(), x.stride(0), C, C
    a.B, a.H, a.W, a.E = B, H, W, E
    a.we, a.be, a.Ntiles, a.Kc = pk.w.data_ptr(), pk.bias.data_ptr(), pk.Ntiles, pk.Kc
    a.wd, a.bd = w.data_ptr(), bias.data_ptr()
    a.k, a.stride, a.act = k, stride, ACT[act]
    a.y, a.y_bs, a.y_ps, a.OH, a.OW = y.data_ptr(), y.stride(0), E, OH, OW
    a.reserved0 = _XD_DBG
    part = None
    if partials:
        nb = int(lib().jabd_expand_dw_nblk(OH, OW, k, stride))
        part = torch.empty((B, nb, E), dtype=torch.float32, device=x.device)
        a.nblk, a.part = nb, part.data_ptr()
    t = None
    if skip is not None:
        t = torch.empty((B, OH, OW, C), dtype=torch.float32, device=x.device)
        a.sw, a.sb = skip[0].data_ptr(), skip[1].data_ptr()
        a.sy, a.sy_bs, a.sy_ps = t.data_ptr(), t.stride(0), C
    if pre is not None:
        ppk, pg, pres, pact = pre
        if (ppk.KH != 1 or ppk.KW != 1 or ppk.Cin != C or ppk.Cout != C or ppk.Cin2 or
                ppk.bias is None or ppk.Kc != 1 or ppk.Ntiles != 1):
            raise ValueError("expand_dw: pre must be a plain Cin -> Cin 1x1 conv with a bias")
        _check("expand_dw.pre.res", pres)
        if tuple(pres.shape) != tuple(x.shape) or pres.stride() != x.stride():
            raise ValueError("expand_dw: the pre residual must have x's shape and strides")
        if pg.shape != (B, C) or not pg.is_contiguous():
            raise ValueError("expand_dw: the pre gate must be a contiguous [B, Cin] tensor")
        a.pw, a.pb, a.pg, a.pres = ppk.w.data_ptr(), ppk.bias.data_ptr(), pg.data_ptr(), \
            pres.data_ptr()
        a.pg_bs, a.pact = pg.stride(0), ACT[pact]
    call("jabd_expand_dw_nhwc_f32", ctypes.byref(a), _stream())
    return (y, part, t) if skip is not None else (y, part)


# pixels per channel-sum block: 64 gives the 64x64 / 32x32 maps 64 / 16 blocks
# per image instead of 16 / 4 (the 32x32 sums ran as 128 workgroups);
# JABD_CSUM_PX=256 restores the old split (A/B)
_CSUM_PX = int(__import__("os").environ.get("JABD_CSUM_PX", "64"))


def channel_sums(x, nblk=None):
    B, H, W, C = x.shape
    HW = H * W
    if nblk is None:
        nblk = max(1, min(64, HW // _CSUM_PX))
    part = torch.empty((B, nblk, C), dtype=torch.float32, device=x.device)
    call("jabd_channel_sum_f32", x.data_ptr(), x.stride(0), C, B, HW, C, nblk, part.data_ptr(),
         _stream())
    return part


def dims3(shape):
    """A tensor shape as the (d0, d1, d2) of jabd_window_copy: conv weights
    [Cout][Cin][KH][KW] -> (Cout, Cin, KH*KW); vectors [C] -> (1, C, 1)."""
    shape = tuple(shape)
    if len(shape) == 0:
        return (1, 1, 1)
    if len(shape) == 1:
        return (1, shape[0], 1)
    if len(shape) == 2:
        return (shape[0], shape[1], 1)
    n2 = 1
    for d in shape[2:]:
        n2 *= d
    return (shape[0], shape[1], n2)


def window_copies(items):
    """[(src, dst, fill[, off2[, scale]])] -> dst (dense) = scale * src's
    window starting at off2 along dim 2, fill outside
    (jabd_window_copy_multi_f32; src None = fill only).  Both tensors are
    read as dims3() boxes, so a pad or a crop along dims 0 / 1 of a conv
    weight or a BN vector, or a column range of a [rows][cols] matrix, is
    one descriptor; up to 32 per launch."""
    from ._lib import WINDOW_MAX, WindowCopy
    for i in range(0, len(items), WINDOW_MAX):
        chunk = items[i:i + WINDOW_MAX]
        arr = (WindowCopy * len(chunk))()
        for d, it in zip(arr, chunk):
            src, dst, fill = it[:3]
            if not dst.is_contiguous() or (src is not None and not src.is_contiguous()):
                raise RuntimeError("window_copies: tensors must be contiguous")
            d.src = src.data_ptr() if src is not None else None
            d.dst = dst.data_ptr()
            d.s0, d.s1, d.s2 = dims3(src.shape) if src is not None else (0, 0, 0)
            d.d0, d.d1, d.d2 = dims3(dst.shape)
            d.off2 = int(it[3]) if len(it) > 3 else 0
            d.fill = float(fill)
            d.scale = float(it[4]) if len(it) > 4 else 1.0
        call("jabd_window_copy_multi_f32", len(chunk), arr, _stream())


def transpose(src, out=None):
    """[rows][cols] -> [cols][rows] on the device (jabd_transpose_f32)."""
    rows, cols = src.shape
    out = torch.empty((cols, rows), dtype=torch.float32, device=src.device) if out is None else out
    call("jabd_transpose_f32", src.data_ptr(), rows, cols, out.data_ptr(), _stream())
    return out


def channel_total(x):
    """Per-channel sum of an NHWC tensor: block partials (jabd_channel_sum_f32)
    summed in a fixed order (jabd_colsum_f32)."""
    part = channel_sums(x)
    C = x.shape[3]
    out = torch.empty(C, dtype=torch.float32, device=x.device)
    call("jabd_colsum_f32", part.data_ptr(), part.shape[0] * part.shape[1], C, out.data_ptr(),
         _stream())
    return out


def eca_gates_multi(xs, w1ds, gate):
    """ECA gates ([B, C] each) of up to 4 NHWC tensors in two launches
    (jabd_eca_pool_gate_multi_f32); the same as eca_gate(channel_sums(x), ...)
    per tensor.  None when a tensor does not qualify (k > 9, C % 4)."""
    n = len(xs)
    if n == 0 or n > 4 or any(w.numel() > 9 or x.shape[3] % 4 for x, w in zip(xs, w1ds)):
        return None
    B = xs[0].shape[0]
    dev = xs[0].device
    A64, A32, AP = ctypes.c_int64 * n, ctypes.c_int32 * n, ctypes.c_void_p * n
    nblk = [max(1, min(64, (x.shape[1] * x.shape[2]) // _CSUM_PX)) for x in xs]
    parts = [torch.empty((B, nb, x.shape[3]), dtype=torch.float32, device=dev)
             for x, nb in zip(xs, nblk)]
    scales = [torch.empty((B, x.shape[3]), dtype=torch.float32, device=dev) for x in xs]
    arrs = (AP(*[x.data_ptr() for x in xs]), A64(*[x.stride(0) for x in xs]),
            A32(*[x.stride(2) for x in xs]), A64(*[x.shape[1] * x.shape[2] for x in xs]),
            A32(*[x.shape[3] for x in xs]), A64(*nblk), AP(*[p.data_ptr() for p in parts]),
            AP(*[w.data_ptr() for w in w1ds]), A32(*[w.numel() for w in w1ds]),
            AP(*[s.data_ptr() for s in scales]))
    a = [ctypes.addressof(t) for t in arrs]
    call("jabd_eca_pool_gate_multi_f32", n, B, a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7],
         a[8], ACT[gate], a[9], _stream())
    return scales


def eca_gate(part, hw, w1d, gate, return_mean=False):
    B, nblk, C = part.shape
    # many tile partials: reduce them over many workgroups first, unless the
    # quad-vectorised gate kernel (C % 4 == 0, k <= 9) spreads the rows itself
    if nblk > 64 and not (C % 4 == 0 and w1d.numel() <= 9 and nblk <= 4096):
        nsplit = min(64, (nblk + 7) // 8)
        red = torch.empty((B, nsplit, C), dtype=torch.float32, device=part.device)
        call("jabd_partial_reduce_f32", part.data_ptr(), nblk, B, C, nsplit, red.data_ptr(),
             _stream())
        part, nblk = red, nsplit
    scale = torch.empty((B, C), dtype=torch.float32, device=part.device)
    mean = torch.empty((B, C), dtype=torch.float32, device=part.device) if return_mean else None
    call("jabd_eca_gate_f32", part.data_ptr(), nblk, B, C, hw, w1d.data_ptr(), w1d.numel(),
         ACT[gate], scale.data_ptr(), _ptr(mean), _stream())
    return (scale, mean) if return_mean else scale


def nlm_fused(src, lateral, nlm_w, sizes, save=False):
    """lateral + NLM(nearest(src -> lateral's size)); all NHWC.  lateral=None
    is the standalone NLM.forward(src) (no up-sample, no add).

    save=True also returns (q, ctx, kpool, vpool) for the backward."""
    B, hs, ws, C = src.shape
    h, w = (hs, ws) if lateral is None else (lateral.shape[1], lateral.shape[2])
    wq, bq, wk, bk, wv, bv, wW, bW = nlm_w
    ch = wq.shape[0]
    S = sum(s * s for s in sizes)
    kp = torch.empty((B, S, ch), dtype=torch.float32, device=src.device)
    vp = torch.empty_like(kp)
    arr = (ctypes.c_int32 * len(sizes))(*sizes)
    kv = torch.empty((B, hs * ws, 2 * ch), dtype=torch.float32, device=src.device)
    call("jabd_nlm_pool_f32", src.data_ptr(), src.stride(0), C, B, hs, ws, C, h, w,
         wk.data_ptr(), bk.data_ptr(), wv.data_ptr(), bv.data_ptr(), ch, arr, len(sizes),
         kp.data_ptr(), vp.data_ptr(), kv.data_ptr(), _stream())
    out = torch.empty((B, h, w, C), dtype=torch.float32, device=src.device)
    q = ctx = None
    if save:
        q = torch.empty((B, h * w, ch), dtype=torch.float32, device=src.device)
        ctx = torch.empty_like(q)
    call("jabd_nlm_apply_f32", src.data_ptr(), src.stride(0), C, B, hs, ws, C, h, w,
         wq.data_ptr(), bq.data_ptr(), kp.data_ptr(), vp.data_ptr(), S, ch, wW.data_ptr(),
         bW.data_ptr(), _ptr(lateral), out.data_ptr(), _ptr(q), _ptr(ctx), _stream())
    if save:
        return out, (q, ctx, kp, vp)
    return out


def upsample_add(src, lateral):
    """lateral + F.interpolate(src, size=lateral's, mode='nearest'), NHWC."""
    _check("upsample_add.src", src)
    B, hs, ws, C = src.shape
    _, h, w, _ = lateral.shape
    out = torch.empty_like(lateral)
    call("jabd_upsample_nearest_add_f32", src.data_ptr(), B, hs, ws, h, w, C, lateral.data_ptr(),
         out.data_ptr(), _stream())
    return out


def maxpool(x, k=3, stride=2, pad=1):
    B, H, W, C = x.shape
    OH = (H + 2 * pad - k) // stride + 1
    OW = (W + 2 * pad - k) // stride + 1
    y = torch.empty((B, OH, OW, C), dtype=torch.float32, device=x.device)
    call("jabd_maxpool_nhwc_f32", x.data_ptr(), B, H, W, C, k, stride, pad, y.data_ptr(),
         _stream())
    return y


def heads(x, wt, bias, loc, conf, landm, a_off, softmax):
    B, H, W, C = x.shape
    A = loc.shape[1]
    call("jabd_heads_f32", x.data_ptr(), x.stride(0), C, B, H * W, C, wt.data_ptr(),
         bias.data_ptr(), A, a_off, 1 if softmax else 0, loc.data_ptr(), conf.data_ptr(),
         landm.data_ptr(), _stream())


def ssh_tail_heads(c33, t, wb, leaky, loc, conf, landm, a_off, softmax):
    """The 40-channel SSH's tail + heads of one level (jabd_ssh_tail_heads_f32):
    c33 = relu(conv3X3) [B,h,w,20], t = leaky(conv5X5_1) [B,h,w,12] -> the
    level's loc / conf / landm rows from anchor a_off."""
    _check("ssh_tail.c33", c33)
    _check("ssh_tail.t", t)
    B, h, w, _ = c33.shape
    if tuple(t.shape) != (B, h, w, 12) or not t.is_contiguous():
        raise ValueError(f"ssh_tail_heads: t must be contiguous [B,h,w,12], got {tuple(t.shape)}")
    call("jabd_ssh_tail_heads_f32", c33.data_ptr(), c33.stride(0), c33.stride(2), t.data_ptr(),
         t.stride(0), B, h, w, wb.data_ptr(), float(leaky), loc.shape[1], a_off,
         1 if softmax else 0, loc.data_ptr(), conf.data_ptr(), landm.data_ptr(), _stream())


def heads_scatter(y, loc, conf, landm, a_off, softmax):
    """y [B, h, w, 32] (the three heads as one 1x1 GEMM) -> loc / conf / landm rows."""
    B, h, w, _ = y.shape
    call("jabd_heads_scatter_f32", y.data_ptr(), B, h * w, loc.shape[1], a_off,
         1 if softmax else 0, loc.data_ptr(), conf.data_ptr(), landm.data_ptr(), _stream())


def adaptive_pool(x, sizes):
    """cat over sizes of AdaptiveAvgPool2d((s, s)) of NHWC x -> [B, S, C]."""
    B, H, W, C = x.shape
    S = sum(s * s for s in sizes)
    out = torch.empty((B, S, C), dtype=torch.float32, device=x.device)
    arr = (ctypes.c_int32 * len(sizes))(*sizes)
    n = int(lib().jabd_adaptive_pool_ws_floats(B, H, C, arr, len(sizes)))
    ws = torch.empty(max(n, 1), dtype=torch.float32, device=x.device)
    call("jabd_adaptive_pool_f32", x.data_ptr(), x.stride(0), B, H, W, C, arr, len(sizes),
         out.data_ptr(), ws.data_ptr(), ws.numel(), _stream())
    return out


def upsample(src, h, w, mode):
    """F.interpolate(src, size=(h, w), mode) on NHWC: 'nearest', or 'bicubic'
    with align_corners=True (train_mobilenetV3_ecagai.py:270,279)."""
    _check("upsample.src", src)
    B, hs, ws, C = src.shape
    out = torch.empty((B, h, w, C), dtype=torch.float32, device=src.device)
    if mode == "nearest":
        call("jabd_upsample_nearest_f32", src.data_ptr(), B, hs, ws, h, w, C, out.data_ptr(),
             _stream())
    elif mode == "bicubic":
        call("jabd_upsample_bicubic_ac_f32", src.data_ptr(), B, hs, ws, C, out.data_ptr(), h, w,
             _stream())
    else:
        raise NotImplementedError(f"up-sampling mode {mode!r}")
    return out


def nlm_attn(q, kp, vp, save=False):
    """softmax(q . kp^T) . vp per pixel: q [B, h, w, ch], kp / vp [B, S, ch] ->
    ctx [B, h, w, ch] (+ lse [B, h*w] when save)."""
    B, h, w, ch = q.shape
    S = kp.shape[1]
    ctx = torch.empty_like(q)
    lse = torch.empty((B, h * w), dtype=torch.float32, device=q.device) if save else None
    call("jabd_nlm_attn_fwd_f32", q.data_ptr(), kp.data_ptr(), vp.data_ptr(), B, h * w, S, ch,
         ctx.data_ptr(), _ptr(lse), _stream())
    return (ctx, lse) if save else ctx


def add3(a, b, c=None, out=None):
    """a + b (+ c), same-shape dense tensors."""
    if out is None:
        out = torch.empty_like(a)
    call("jabd_add3_f32", a.data_ptr(), b.data_ptr(), _ptr(c), a.numel(), out.data_ptr(),
         _stream())
    return out
