"""Microbenchmark of single conv launches at the C2 / R50 layer shapes.

Each shape runs with the library's current kernel choice (set JABD_CONV32 /
JABD_CONV_GENERIC in the environment for A/B), checks the output against a
torch fp32 reference on the GPU (max-abs error / max-abs ref), and prints
us / TFLOP/s / algorithmic GB/s (input, skip source, residual, weights,
output) and the roofline time max(FLOP/157.3T, bytes/8T).

  python3 tools/convbench.py [--set mnv3|r50|all] [--reps 20]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]
from jabd_amd import functional as F  # noqa: E402

# (name, B, H, W, Cin, Cout, k, stride, x2 channels (0 = none), ascale, res, act)
MNV3 = [
    ("b1.proj", 32, 512, 512, 16, 16, 1, 1, 0, 1, 1, "relu"),
    ("b2.proj", 32, 256, 256, 64, 24, 1, 1, 16, 1, 0, "relu"),
    ("b3.proj", 32, 256, 256, 72, 24, 1, 1, 0, 1, 1, "relu"),
    ("b4.proj", 32, 128, 128, 72, 40, 1, 1, 24, 1, 0, "relu"),
    ("b5.proj", 32, 128, 128, 120, 40, 1, 1, 0, 1, 1, "relu"),
    ("b7.proj", 32, 64, 64, 240, 80, 1, 1, 40, 1, 0, "hswish"),
    ("b8.proj", 32, 64, 64, 200, 80, 1, 1, 0, 1, 1, "hswish"),
    ("b11.proj", 32, 64, 64, 480, 112, 1, 1, 80, 1, 0, "hswish"),
    ("b12.proj", 32, 64, 64, 672, 112, 1, 1, 0, 1, 1, "hswish"),
    ("b13.proj", 32, 32, 32, 672, 160, 1, 1, 112, 1, 0, "hswish"),
    ("b14.proj", 32, 32, 32, 672, 160, 1, 1, 0, 1, 1, "hswish"),
    ("b15.proj", 32, 32, 32, 960, 160, 1, 1, 0, 1, 1, "hswish"),
    ("b12.exp", 32, 64, 64, 112, 672, 1, 1, 0, 0, 0, "hswish"),
    ("b15.exp", 32, 32, 32, 160, 960, 1, 1, 0, 0, 0, "hswish"),
    ("fpn.lat1", 32, 128, 128, 40, 40, 1, 1, 0, 1, 0, "leaky"),
    ("ssh1.c3", 32, 128, 128, 40, 20, 3, 1, 0, 1, 0, "relu"),
    ("merge1", 32, 128, 128, 40, 40, 3, 1, 0, 0, 0, "leaky"),
]
# training-pass 1x1 data gradients (transposed weights, no act) at C4 shapes
TR = [
    ("b1.proj", 32, 512, 512, 16, 16, 1, 1, 0, 1, 1, "relu"),
    ("b1e.dg", 32, 512, 512, 64, 16, 1, 1, 0, 0, 0, "none"),
    ("b3e.dg", 32, 256, 256, 72, 24, 1, 1, 0, 0, 0, "none"),
    ("b5e.dg", 32, 128, 128, 120, 40, 1, 1, 0, 0, 0, "none"),
    ("b1p.dg", 32, 512, 512, 16, 16, 1, 1, 0, 0, 0, "none"),
    ("b3p.dg", 32, 256, 256, 24, 72, 1, 1, 0, 0, 0, "none"),
    ("b12.p.asc", 32, 64, 64, 672, 112, 1, 1, 0, 1, 1, "hswish"),
    ("b12.p.noasc", 32, 64, 64, 672, 112, 1, 1, 0, 0, 1, "hswish"),
    ("b11.p.asc", 32, 64, 64, 480, 112, 1, 1, 80, 1, 0, "hswish"),
    ("b11.p.noasc", 32, 64, 64, 480, 112, 1, 1, 80, 0, 0, "hswish"),
    ("b15.p.asc", 32, 32, 32, 960, 160, 1, 1, 0, 1, 1, "hswish"),
    ("b15.p.noasc", 32, 32, 32, 960, 160, 1, 1, 0, 0, 1, "hswish"),
    ("t.480a", 3, 32, 48, 112, 480, 1, 1, 0, 0, 0, "none"),
    ("t.480b", 3, 20, 24, 112, 480, 1, 1, 0, 0, 0, "none"),
    ("t.480c", 2, 32, 32, 112, 480, 1, 1, 0, 0, 0, "none"),
    ("t.480d", 3, 32, 48, 480, 112, 1, 1, 0, 0, 0, "none"),
    ("t.480e", 3, 32, 48, 112, 480, 1, 1, 0, 1, 0, "none"),
]
R50 = [
    ("l1.c1", 16, 256, 256, 64, 64, 1, 1, 0, 0, 0, "relu"),
    ("l1.c2", 16, 256, 256, 64, 64, 3, 1, 0, 0, 0, "relu"),
    ("l1.c3", 16, 256, 256, 64, 256, 1, 1, 64, 0, 0, "relu"),
    ("l1.c1b", 16, 256, 256, 256, 64, 1, 1, 0, 0, 0, "relu"),
    ("l2.c1a", 16, 256, 256, 256, 128, 1, 1, 0, 0, 0, "relu"),
    ("l2.c1", 16, 128, 128, 512, 128, 1, 1, 0, 0, 0, "relu"),
    ("l2.c2", 16, 128, 128, 128, 128, 3, 1, 0, 0, 0, "relu"),
    ("l2.c3", 16, 128, 128, 128, 512, 1, 1, 0, 0, 1, "relu"),
    ("l3.c1", 16, 64, 64, 1024, 256, 1, 1, 0, 0, 0, "relu"),
    ("l3.c2", 16, 64, 64, 256, 256, 3, 1, 0, 0, 0, "relu"),
    ("l3.c3", 16, 64, 64, 256, 1024, 1, 1, 0, 0, 1, "relu"),
    ("l4.c1", 16, 32, 32, 2048, 512, 1, 1, 0, 0, 0, "relu"),
    ("l4.c2", 16, 32, 32, 512, 512, 3, 1, 0, 0, 0, "relu"),
    ("l4.c3", 16, 32, 32, 512, 2048, 1, 1, 0, 0, 1, "relu"),
    ("l2.c2s2", 16, 256, 256, 128, 128, 3, 2, 0, 0, 0, "relu"),
    ("l4.c2s2", 16, 64, 64, 512, 512, 3, 2, 0, 0, 0, "relu"),
    ("l3.c2as", 16, 64, 64, 256, 256, 3, 1, 0, 1, 0, "relu"),
]
# C3 (R50 training, bs64 1024^2) short-K / narrow 1x1 forwards (no bias / act)
R50T = [
    ("t.l1.c3", 64, 256, 256, 64, 256, 1, 1, 0, 0, 0, "none"),
    ("t.l1.c1", 64, 256, 256, 256, 64, 1, 1, 0, 0, 0, "none"),
    ("t.l2.c3", 64, 128, 128, 128, 512, 1, 1, 0, 0, 0, "none"),
    ("t.l2.c1", 64, 128, 128, 512, 128, 1, 1, 0, 0, 0, "none"),
    ("t.l3.c3", 64, 64, 64, 256, 1024, 1, 1, 0, 0, 0, "none"),
    ("t.l1.c2", 64, 256, 256, 64, 64, 3, 1, 0, 0, 0, "none"),
]


def ref(x, w2d, bias, k, stride, x2, sc, res, act):
    xs = x * sc[:, None, None, :] if sc is not None else x
    xn = xs.permute(0, 3, 1, 2)
    cout = w2d.shape[1]
    cin = x.shape[3]
    wt = w2d[:k * k * cin].reshape(k, k, cin, cout).permute(3, 2, 0, 1)
    y = torch.nn.functional.conv2d(xn, wt, None, stride, k // 2)
    if x2 is not None:
        y = y + torch.nn.functional.conv2d(x2.permute(0, 3, 1, 2),
                                           w2d[k * k * cin:].t()[:, :, None, None])
    y = y.permute(0, 2, 3, 1) + bias
    if res is not None:
        y = y + res
    if act == "relu":
        y = torch.relu(y)
    elif act == "leaky":
        y = torch.nn.functional.leaky_relu(y, 0.1)
    elif act == "hswish":
        y = torch.nn.functional.hardswish(y)
    return y


def run(shape, reps):
    name, B, H, W, cin, cout, k, stride, c2, asc, hasres, act = shape
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, H, W, cin, device=dev, generator=g)
    x2 = torch.randn(B, H, W, c2, device=dev, generator=g) if c2 else None
    K = k * k * cin + c2
    w2d = torch.randn(K, cout, device=dev, generator=g) / K ** 0.5
    bias = torch.randn(cout, device=dev, generator=g)
    sc = torch.rand(B, cin, device=dev, generator=g) if asc else None
    OH, OW = (H - 1) // stride + 1, (W - 1) // stride + 1
    res = torch.randn(B, OH, OW, cout, device=dev, generator=g) if hasres else None
    pk = F.PackedConv(w2d, bias, k, k, cin, c2)
    kw = dict(stride=stride, pad=k // 2, act=act, slope=0.1, ascale=sc, x2=x2, res=res)
    y = F.conv(x, pk, **kw)
    F._CONV_DBG = int(os.environ.get("CONV_DBG", "0"))
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    r = ref(x, w2d, bias, k, stride, x2, sc, res, act)
    err = float((y - r).abs().max() / r.abs().max())
    for _ in range(3):
        F.conv(x, pk, **kw)
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        F.conv(x, pk, **kw)
    e.record()
    torch.cuda.synchronize()
    t = s.elapsed_time(e) / reps * 1e3
    M = B * OH * OW
    fl = 2.0 * M * K * cout
    nb = 4.0 * (x.numel() + (x2.numel() if c2 else 0) + (res.numel() if hasres else 0)
                + K * cout + M * cout)
    roof = max(fl / 157.3e12, nb / 8e12) * 1e6
    tl = ""
    if k == 1 and not c2 and not asc and os.environ.get("CB_TORCH"):
        a2, w2 = x.reshape(-1, cin), w2d.contiguous()
        torch.mm(a2, w2)
        s.record()
        for _ in range(reps):
            torch.mm(a2, w2)
        e.record()
        torch.cuda.synchronize()
        tl = "  torch.mm %7.1f us" % (s.elapsed_time(e) / reps * 1e3)
    print("%-9s M%8d K%5d N%5d k%d  %8.1f us  %6.1f TF  %6.0f GB/s  roof %7.1f (%3.0f%%)  err %.1e"
          % (name, M, K, cout, k, t, fl / t / 1e6, nb / t / 1e3, roof, 100 * roof / t, err)
          + tl, flush=True)
    return t, roof, err


# expand 1x1 + depthwise (fused kernel): (name, B, H, W, Cin, E, k, stride, act)
XD = [
    ("b1.xd", 32, 512, 512, 16, 16, 3, 1, "relu"),
    ("b2.xd", 32, 512, 512, 16, 64, 3, 2, "relu"),
    ("b3.xd", 32, 256, 256, 24, 72, 3, 1, "relu"),
    ("b4.xd", 32, 256, 256, 24, 72, 5, 2, "relu"),
    ("b5.xd", 32, 128, 128, 40, 120, 5, 1, "relu"),
    ("b7.xd", 32, 128, 128, 40, 240, 3, 2, "hswish"),
    ("b8.xd", 32, 64, 64, 80, 200, 3, 1, "hswish"),
    ("b11.xd", 32, 64, 64, 80, 480, 3, 1, "hswish"),
    ("b12.xd", 32, 64, 64, 112, 672, 3, 1, "hswish"),
    ("b13.xd", 32, 64, 64, 112, 672, 5, 2, "hswish"),
    ("b14.xd", 32, 32, 32, 160, 672, 5, 1, "hswish"),
    ("b15.xd", 32, 32, 32, 160, 960, 5, 1, "hswish"),
]


def run_xd(shape, reps):
    name, B, H, W, cin, E, k, stride, act = shape
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, H, W, cin, device=dev, generator=g)
    we = torch.randn(cin, E, device=dev, generator=g) / cin ** 0.5
    be = torch.randn(E, device=dev, generator=g) * 0.1
    wd = torch.randn(k * k, E, device=dev, generator=g) / k
    bd = torch.randn(E, device=dev, generator=g) * 0.1
    pk = F.PackedConv(we, be, 1, 1, cin)
    # XD_SKIP_BRANCH=1: stride-2 layers carry the block's fused dw3x3/s2 skip
    # branch, as in the C2 forward (nets/mobilenetV3.py:126-137)
    skip = None
    if stride == 2 and os.environ.get("XD_SKIP_BRANCH") == "1":
        skip = (torch.randn(9, cin, device=dev, generator=g) / 3,
                torch.randn(cin, device=dev, generator=g) * 0.1)
    y, part = F.expand_dw(x, pk, wd, bd, k, stride, act=act, skip=skip)[:2]
    dbg = int(os.environ.get("XD_DBG", "0"))
    if dbg:
        F._XD_DBG = dbg
    fa = torch.relu if act == "relu" else torch.nn.functional.hardswish
    e1 = fa(x.reshape(-1, cin) @ we + be).reshape(B, H, W, E).permute(0, 3, 1, 2)
    r = torch.nn.functional.conv2d(e1, wd.t().reshape(E, 1, k, k), bd, stride, k // 2, 1, E)
    r = fa(r).permute(0, 2, 3, 1)
    err = float((y - r).abs().max() / r.abs().max())
    perr = float((part.sum(1) - r.sum((1, 2))).abs().max() / r.sum((1, 2)).abs().max())
    for _ in range(3):
        F.expand_dw(x, pk, wd, bd, k, stride, act=act, skip=skip)
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        F.expand_dw(x, pk, wd, bd, k, stride, act=act, skip=skip)
    e.record()
    torch.cuda.synchronize()
    t = s.elapsed_time(e) / reps * 1e3
    fl = 2.0 * B * H * W * cin * E + 2.0 * y.numel() * k * k
    nb = 4.0 * (x.numel() + y.numel())
    roof = max(fl / 157.3e12, nb / 8e12) * 1e6
    print("%-9s %4dx%-4d %4d->%-4d k%d s%d  %8.1f us  %6.1f TF  %6.0f GB/s  roof %7.1f (%3.0f%%)  "
          "err %.1e part %.1e" % (name, H, W, cin, E, k, stride, t, fl / t / 1e6, nb / t / 1e3,
                                  roof, 100 * roof / t, err, perr), flush=True)
    return t, roof, max(err, perr)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", default="mnv3")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    shapes = {"tr": TR, "mnv3": MNV3, "r50": R50, "r50t": R50T, "all": MNV3 + R50, "xd": XD}[args.set]
    if args.only:
        shapes = [s for s in shapes if s[0] in args.only.split(",")]
    print("# JABD_CONV32=%s JABD_CONV_GENERIC=%s" % (os.environ.get("JABD_CONV32"),
                                                    os.environ.get("JABD_CONV_GENERIC")))
    bad = 0
    for sh in shapes:
        _, _, err = (run_xd if args.set == "xd" else run)(sh, args.reps)
        bad += err > 1e-4
    print("# errors > 1e-4:", bad)


if __name__ == "__main__":
    main()
