"""Depthwise weight-gradient timing at the C4 (MNv3 1024^2 bs32) 3x3 layer
shapes: jabd_dw_wgrad_f32 / _bnin_f32 (train.hip), us per call and GB/s of
x + dy read once.  JABD_DW_WGRAD_ROWS=0 selects the strip kernel for A/B.

  python3 tools/dwwg_bench.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]
from jabd_amd._lib import lib  # noqa: E402

SHAPES = [  # name, B, H, W, C, stride, bnin
    ("b1.dw s2 bnin", 32, 512, 512, 64, 2, True),
    ("b2.dw", 32, 256, 256, 72, 1, False),
    ("b3.dw s2", 32, 256, 256, 72, 2, False),
    ("b6.dw s2", 32, 128, 128, 240, 2, False),
    ("b7.dw", 32, 64, 64, 200, 1, False),
    ("b8.dw", 32, 64, 64, 184, 1, False),
    ("b10.dw", 32, 64, 64, 480, 1, False),
]


def main():
    dev = torch.device("cuda")
    L = lib()
    for name, B, H, W, C, s, bnin in SHAPES:
        OH, OW = (H - 1) // s + 1, (W - 1) // s + 1
        x = torch.randn(B, H, W, C, device=dev)
        dy = torch.randn(B, OH, OW, C, device=dev)
        part = torch.empty(int(L.jabd_dw_wgrad_part_floats(B * OH * OW, C, 3)), device=dev)
        dw = torch.empty(C, 9, device=dev)
        mean, inv, gam, bet = (torch.rand(C, device=dev) for _ in range(4))

        def run():
            if bnin:
                r = L.jabd_dw_wgrad_bnin_f32(x.data_ptr(), dy.data_ptr(), B, H, W, C, OH, OW, 3, s, 1,
                                             mean.data_ptr(), inv.data_ptr(), gam.data_ptr(),
                                             bet.data_ptr(), 1, 0.0, part.data_ptr(), dw.data_ptr(), None)
            else:
                r = L.jabd_dw_wgrad_f32(x.data_ptr(), dy.data_ptr(), B, H, W, C, OH, OW, 3, s, 1,
                                        part.data_ptr(), dw.data_ptr(), None)
            assert r == 0
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 10 * 1e3
        gb = (x.numel() + dy.numel()) * 4 / 1e9
        print(f"{name:16s} {us:8.1f} us  {gb / us * 1e6:7.0f} GB/s")


if __name__ == "__main__":
    main()
