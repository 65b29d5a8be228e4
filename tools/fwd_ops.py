"""Per-op timing of one C2 forward (bs32 1024^2 JABD-MNv3 eval) with HIP events
around every jabd functional call on the launch stream.  Prints each launch
with its algorithmic FLOP / bytes and the roofline time max(FLOP/157.3T,
bytes/8T), then a per-op-kind summary.

  python3 tools/fwd_ops.py [--kind mnv3|r50] [--batch 32] [--size 1024]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]
import bench  # noqa: E402
from jabd_amd import engine, functional as F, synth  # noqa: E402

PEAK, BW = 157.3e12, 8e12


def _nb(*ts):
    return 4.0 * sum(t.numel() for t in ts if isinstance(t, torch.Tensor))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="mnv3")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=1024)
    args = ap.parse_args()
    dev = torch.device("cuda")
    if args.kind == "mnv3":
        m = bench.build_model(dev)
    else:
        from nets.retinaface_eca_nonlocal import RetinaFace
        from nets.retinaface_training import weights_init
        from utils.config import cfg_re50
        m = RetinaFace(cfg=cfg_re50, mode="eval")
        weights_init(m)
        m = m.to(dev).eval()
    x = synth.images(args.batch, args.size, device=dev)
    with torch.no_grad():
        for _ in range(3):
            m(x)
    torch.cuda.synchronize()
    recs = []

    def wrap(name, fn, cost):
        def w(*a, **kw):
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            o = fn(*a, **kw)
            e.record()
            fl, nb, desc = cost(o, *a, **kw)
            recs.append((name, s, e, fl, nb, desc))
            return o
        return w

    def c_conv(o, xx, pk, stride=1, pad=0, **kw):
        M = o.shape[0] * o.shape[1] * o.shape[2]
        K = pk.KH * pk.KW * pk.Cin + pk.Cin2
        nb = _nb(xx, kw.get("x2")) + 4.0 * (K * pk.Cout + M * pk.Cout)
        return 2.0 * M * K * pk.Cout, nb, "M%d K%d N%d k%d s%d" % (M, K, pk.Cout, pk.KH, stride)

    def c_xd(o, xx, pk, w, b, k, stride, **kw):
        y = o[0]
        M = y.shape[0] * y.shape[1] * y.shape[2]
        E = y.shape[3]
        Min = xx.shape[0] * xx.shape[1] * xx.shape[2]
        fl = 2.0 * Min * pk.Cin * E + 2.0 * M * E * k * k
        nb = _nb(xx, y)
        pre = kw.get("pre")
        if pre is not None:   # the previous block's project fused in front
            fl += 2.0 * Min * pre[0].Cin * pre[0].Cout
            nb += _nb(pre[2])
        return fl, nb, "Min%d Cin%d E%d k%d s%d%s" % (Min, pk.Cin, E, k, stride,
                                                      " +proj" if pre is not None else "")

    def c_dw(o, xx, w, b, k, stride, **kw):
        y = o[0]
        M = y.shape[0] * y.shape[1] * y.shape[2]
        return 2.0 * M * y.shape[3] * k * k, _nb(xx, y), "C%d k%d s%d" % (y.shape[3], k, stride)

    def c_generic(o, *a, **kw):
        ins = [t for t in a if isinstance(t, torch.Tensor)]
        outs = o if isinstance(o, tuple) else (o,)
        return 0.0, _nb(*ins) + _nb(*outs), "x".join(str(s) for s in ins[0].shape) if ins else ""

    def c_tail(o, c33, t, wb, leaky, loc, *a, **kw):
        # conv7X7_2 on the tile + halo counted on the tile only (algorithmic),
        # conv5X5_2, conv7x7_3 (90 -> 10 each) and the heads (40 -> 32)
        M = c33.shape[0] * c33.shape[1] * c33.shape[2]
        fl = 2.0 * M * (3 * 90 * 10 + 40 * 32)
        nb = _nb(c33, t) + 4.0 * M * 32
        return fl, nb, "M%d (3x 90->10, heads 40->32)" % M

    F.conv = wrap("conv", F.conv, c_conv)
    F.ssh_tail_heads = wrap("ssh_tail", F.ssh_tail_heads, c_tail)
    F.expand_dw = wrap("expand_dw", F.expand_dw, c_xd)
    F.dwconv = wrap("dwconv", F.dwconv, c_dw)
    for n in ("stem", "channel_sums", "eca_gate", "nlm_fused", "maxpool", "heads"):
        setattr(F, n, wrap(n, getattr(F, n), c_generic))
    s0 = torch.cuda.Event(enable_timing=True)
    e0 = torch.cuda.Event(enable_timing=True)
    with torch.no_grad():
        s0.record()
        m(x)
        e0.record()
    torch.cuda.synchronize()
    tot = s0.elapsed_time(e0) * 1e3
    kinds = {}
    for name, s, e, fl, nb, desc in recs:
        t = s.elapsed_time(e) * 1e3
        roof = max(fl / PEAK, nb / BW) * 1e6
        k = kinds.setdefault(name, [0, 0.0, 0.0, 0.0, 0.0])
        k[0] += 1; k[1] += t; k[2] += roof; k[3] += fl; k[4] += nb
        print("%-12s %-36s %8.1f us  %6.1f TF  %6.0f GB/s  roof %7.1f us (%3.0f%%)"
              % (name, desc, t, fl / t / 1e6, nb / t / 1e3, roof, 100 * roof / t))
    print("\nforward wall %.1f us; sum of op events %.1f us" % (tot, sum(v[1] for v in kinds.values())))
    for name, (n, t, roof, fl, nb) in sorted(kinds.items(), key=lambda kv: -kv[1][1]):
        print("%-12s n=%3d  %8.1f us  roof %8.1f us  (%3.0f%%)  %6.1f TF  %6.0f GB/s"
              % (name, n, t, roof, 100 * roof / t, fl / t / 1e6, nb / t / 1e3))


if __name__ == "__main__":
    main()
