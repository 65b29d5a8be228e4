"""Weight-gradient microbenchmark at the R50 / MNv3 training shapes: jabd
conv wgrad vs float64-free torch reference (torch.nn.grad.conv2d_weight on
GPU fp32); prints us, TFLOP/s and the max relative error.

  JABD_WGRAD32=0|1 python3 tools/wgradbench.py
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]
from jabd_amd import train as T  # noqa: E402

SHAPES = [  # name, B, H, W, Cin, Cout, k, stride
    ("l1.c1", 64, 256, 256, 64, 64, 1, 1),
    ("l1.c2", 64, 256, 256, 64, 64, 3, 1),
    ("l1.c3", 64, 256, 256, 64, 256, 1, 1),
    ("l2.c1", 64, 256, 256, 256, 128, 1, 1),
    ("l2.c2", 64, 256, 256, 128, 128, 3, 2),
    ("l2.c3", 64, 128, 128, 128, 512, 1, 1),
    ("l3.c2", 64, 64, 64, 256, 256, 3, 1),
    ("l3.c3", 64, 64, 64, 256, 1024, 1, 1),
    ("l4.c2", 64, 32, 32, 512, 512, 3, 1),
    ("l4.c3", 64, 32, 32, 512, 2048, 1, 1),
    ("mb.exp", 32, 64, 64, 112, 672, 1, 1),
    ("mb.proj", 32, 64, 64, 672, 112, 1, 1),
]


def main():
    dev = torch.device("cuda")
    for name, B, H, W, cin, cout, k, s in SHAPES:
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(B, H, W, cin, device=dev, generator=g)
        OH, OW = (H + 2 * (k // 2) - k) // s + 1, (W + 2 * (k // 2) - k) // s + 1
        dy = torch.randn(B, OH, OW, cout, device=dev, generator=g)
        w = torch.empty(cout, cin, k, k, device=dev)
        dw = T._wgrad(x, dy, w, s, k // 2)
        ref = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2), w.shape, dy.permute(0, 3, 1, 2),
                                          s, k // 2)
        err = float((dw - ref).abs().max() / ref.abs().max())
        torch.cuda.synchronize()
        st = torch.cuda.Event(enable_timing=True)
        en = torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(5):
            T._wgrad(x, dy, w, s, k // 2)
        en.record()
        torch.cuda.synchronize()
        t = st.elapsed_time(en) / 5 * 1e3
        fl = 2.0 * B * OH * OW * cin * k * k * cout
        print("%-8s K%5d N%5d M%9d  %9.1f us  %6.1f TF  err %.1e" % (
            name, cin * k * k, cout, B * OH * OW, t, fl / t / 1e6, err), flush=True)
        del x, dy, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
