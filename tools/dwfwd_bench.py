"""Depthwise training-forward timing (jabd_dwconv_stats_f32 / _bnin_stats_f32:
the conv + its output's BatchNorm statistics) at the C4 (MNv3 1024^2 bs32)
3x3 layer shapes, with the outputs and statistics partials checked against
the strip kernel (JABD_DW_ROWS=0 in a second run, compared through saved
files).

  python3 tools/dwfwd_bench.py [--save out.pt] [--ref ref.pt]
"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]
from jabd_amd._lib import lib, DwArgs  # noqa: E402

SHAPES = [  # name, B, H, W, C, stride, bnin
    ("b1.dw s2 bnin", 32, 512, 512, 64, 2, True),
    ("b2.dw", 32, 256, 256, 72, 1, False),
    ("b3.dw s2 bnin", 32, 256, 256, 72, 2, True),
    ("b6.dw s2 bnin", 32, 128, 128, 240, 2, True),
    ("b7.dw", 32, 64, 64, 200, 1, False),
    ("b10.dw", 32, 64, 64, 480, 1, False),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--save", default="")
    ap.add_argument("--ref", default="")
    a = ap.parse_args()
    dev = torch.device("cuda")
    L = lib()
    saved = {}
    ref = torch.load(a.ref, weights_only=True) if a.ref else None
    for name, B, H, W, C, s, bnin in SHAPES:
        OH, OW = (H - 1) // s + 1, (W - 1) // s + 1
        g = torch.Generator(device=dev).manual_seed(C + s)
        x = torch.randn(B, H, W, C, device=dev, generator=g)
        wt = torch.randn(9, C, device=dev, generator=g) / 3
        y = torch.empty(B, OH, OW, C, device=dev)
        nblk = int(L.jabd_dwconv_stats_nblk(B, OH, OW, C))
        part = torch.zeros(nblk, 2, C, device=dev)
        shift = torch.empty(C, device=dev)
        mean, inv = torch.randn(C, device=dev, generator=g), torch.rand(C, device=dev, generator=g) + 0.5
        gam, bet = torch.randn(C, device=dev, generator=g), torch.randn(C, device=dev, generator=g)
        ar = DwArgs()
        ar.x, ar.x_bs, ar.x_ps = x.data_ptr(), x.stride(0), C
        ar.B, ar.H, ar.W, ar.C = B, H, W, C
        ar.w, ar.bias = wt.data_ptr(), None
        ar.y, ar.y_bs, ar.y_ps = y.data_ptr(), y.stride(0), C
        ar.OH, ar.OW, ar.k, ar.stride, ar.pad, ar.act = OH, OW, 3, s, 1, 0

        def run():
            if bnin:
                r = L.jabd_dwconv_bnin_stats_f32(ctypes.byref(ar), mean.data_ptr(), inv.data_ptr(),
                                                 gam.data_ptr(), bet.data_ptr(), 3, 0.0,
                                                 part.data_ptr(), shift.data_ptr(), None)
            else:
                r = L.jabd_dwconv_stats_f32(ctypes.byref(ar), part.data_ptr(), shift.data_ptr(), None)
            assert r == 0
        run()
        torch.cuda.synchronize()
        tot = part.double().sum(0)
        if a.save:
            saved[name] = (y[:2].cpu(), tot.cpu(), shift.cpu())
        if ref is not None:
            ry, rt, rs = ref[name]
            same = torch.equal(ry, y[:2].cpu()) and torch.equal(rs, shift.cpu())
            st_err = float(((tot.cpu() - rt).abs() / (rt.abs() + 1.0)).max())
            print(f"{name}: outputs {'bit-identical' if same else 'DIFFER'}; stats rel err {st_err:.2e}")
        for _ in range(2):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(10):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 10 * 1e3
        gb = (x.numel() + y.numel()) * 4 / 1e9
        print(f"{name:16s} {us:8.1f} us  {gb / us * 1e6:7.0f} GB/s")
    if a.save:
        torch.save(saved, a.save)


if __name__ == "__main__":
    main()
