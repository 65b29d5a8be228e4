"""Depthwise data gradient + BatchNorm backward timing (jabd_dw_dgrad_bn_bwd_f32,
train.hip) at the C4 3x3 shapes, in both forms the training graph uses (de
stored, or the two-pass form with de recomputed); JABD_DW_DGRAD_ROWS=0 selects
the strip-row kernel for A/B, and --save / --ref compare the outputs bit for
bit across the two runs.

  python3 tools/dwbwd_bench.py [--save f.pt] [--ref f.pt]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]
from jabd_amd._lib import lib  # noqa: E402

SHAPES = [  # name, B, H, W, C, stride, recompute (dz not stored)
    ("b1 s2", 32, 512, 512, 64, 2, True),
    ("b2", 32, 256, 256, 72, 1, False),
    ("b3 s2", 32, 256, 256, 72, 2, True),
    ("b7", 32, 64, 64, 200, 1, False),
    ("b10", 32, 64, 64, 480, 1, False),
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
    for name, B, H, W, C, s, rec in SHAPES:
        OH, OW = (H - 1) // s + 1, (W - 1) // s + 1
        g = torch.Generator(device=dev).manual_seed(C + s)
        dy = torch.randn(B, OH, OW, C, device=dev, generator=g)
        wt = torch.randn(9, C, device=dev, generator=g) / 3
        x = torch.randn(B, H, W, C, device=dev, generator=g)
        mean, inv = torch.randn(C, device=dev, generator=g), torch.rand(C, device=dev, generator=g) + 0.5
        gam, bet = torch.randn(C, device=dev, generator=g), torch.randn(C, device=dev, generator=g)
        part = torch.empty(int(L.jabd_dw_dgrad_bn_part_floats(B, H, W, C)), device=dev)
        dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
        dz = None if rec else torch.empty_like(x)
        dx = torch.empty_like(x)

        def run():
            r = L.jabd_dw_dgrad_bn_bwd_f32(dy.data_ptr(), wt.data_ptr(), B, H, W, C, OH, OW, 3, s, 1,
                                           x.data_ptr(), mean.data_ptr(), inv.data_ptr(),
                                           gam.data_ptr(), bet.data_ptr(), 3, 0.0, part.data_ptr(),
                                           dg.data_ptr(), db.data_ptr(),
                                           dz.data_ptr() if dz is not None else None,
                                           dx.data_ptr(), None)
            assert r == 0
        run()
        torch.cuda.synchronize()
        if a.save:
            saved[name] = (dx[:1].cpu(), dg.cpu(), db.cpu())
        if ref is not None:
            rx, rg, rb = ref[name]
            same = torch.equal(rx, dx[:1].cpu())
            e = max(float(((dg.cpu() - rg).abs() / (rg.abs() + 1)).max()),
                    float(((db.cpu() - rb).abs() / (rb.abs() + 1)).max()))
            print(f"{name}: dx {'bit-identical' if same else 'DIFFER'}; dgamma/dbeta rel err {e:.2e}")
        for _ in range(2):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(10):
            run()
        e1.record()
        torch.cuda.synchronize()
        print(f"{name:8s} {e0.elapsed_time(e1) / 10 * 1e3:8.1f} us")
    if a.save:
        torch.save(saved, a.save)


if __name__ == "__main__":
    main()
