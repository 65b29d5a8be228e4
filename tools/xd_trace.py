"""Workgroup phase timeline of the fused expand+depthwise kernel
(expdw1_kernel built with -DXD_TRACE=1, tools/xd_variant.sh trace
"-DXD_TRACE=1"):

  JABD_LIB=abx/libjabd_trace.so python3 tools/xd_trace.py [--only b2.xd,b4.xd]

Per layer: kernel span (device realtime), workgroups, mean live workgroups
per CU, and per-phase shader-clock cycles of wave 0 (decode -> first input
stage in LDS, expand MFMA loop, epilogue + barrier, depthwise, ECA reduce).
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]
from jabd_amd import functional as F  # noqa: E402
from jabd_amd._lib import lib  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import convbench  # noqa: E402  (tools/)

NCU = 256


def trace(shape, buf):
    name, B, H, W, cin, E, k, stride, act = shape
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, H, W, cin, device=dev, generator=g)
    we = torch.randn(cin, E, device=dev, generator=g) / cin ** 0.5
    be = torch.randn(E, device=dev, generator=g) * 0.1
    wd = torch.randn(k * k, E, device=dev, generator=g) / k
    bd = torch.randn(E, device=dev, generator=g) * 0.1
    pk = F.PackedConv(we, be, 1, 1, cin)
    for _ in range(3):
        F.expand_dw(x, pk, wd, bd, k, stride, act=act)
    torch.cuda.synchronize()
    buf.zero_()
    lib().jabd_xd_trace_set(ctypes.c_void_p(buf.data_ptr()))
    F.expand_dw(x, pk, wd, bd, k, stride, act=act)
    torch.cuda.synchronize()
    lib().jabd_xd_trace_set(ctypes.c_void_p(0))
    t = buf.cpu().numpy().reshape(-1, 8)
    t = t[t[:, 0] != 0].astype(np.float64)
    rt0, rt1 = t[:, 0], t[:, 7]
    span = (rt1.max() - rt0.min()) * 10e-3                  # us (100 MHz)
    life_rt = (rt1 - rt0) * 10e-3
    cyc = t[:, 6] - t[:, 1]
    mhz = float(np.median(cyc / np.maximum(life_rt, 1e-3)))
    ph = {"load": t[:, 2] - t[:, 1], "mfma": t[:, 3] - t[:, 2], "epi": t[:, 4] - t[:, 3],
          "dw": t[:, 5] - t[:, 4], "eca": t[:, 6] - t[:, 5]}
    live = life_rt.sum() / span / NCU
    start = np.sort(rt0 - rt0.min()) * 10e-3
    ramp = start[min(len(start) - 1, NCU * 2)]
    print(f"{name:8s} span {span:7.1f} us  WGs {len(t):6d}  live/CU {live:4.2f}  "
          f"WG life {np.median(life_rt):6.2f} us (p90 {np.percentile(life_rt, 90):6.2f})  "
          f"clk {mhz:5.0f} MHz  first {2 * NCU} WGs started by {ramp:5.2f} us")
    print("          cycles median / p90: " + "  ".join(
        f"{k} {np.median(v):6.0f}/{np.percentile(v, 90):6.0f}" for k, v in ph.items()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    shapes = convbench.XD
    if a.only:
        shapes = [s for s in shapes if s[0] in a.only.split(",")]
    buf = torch.zeros(400000 * 8, dtype=torch.int64, device="cuda")
    for sh in shapes:
        trace(sh, buf)


if __name__ == "__main__":
    main()
