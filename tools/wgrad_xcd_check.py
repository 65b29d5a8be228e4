"""Weight gradients of the C3 / C4 shapes saved for a bit-identity check
between two builds / settings (JABD_WGRAD_XCD=0|1), plus an fp32 GEMM
reference for the 1x1 shapes (x^T dy via torch.mm in row chunks, fp64
accumulation of the chunks).

  python3 tools/wgrad_xcd_check.py OUT.pt [--ref]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]
import torch  # noqa: E402
from jabd_amd import train as T  # noqa: E402

SHAPES = [  # name, B, H, W, Cin, Cout, k, stride
    ("l1.c3", 64, 256, 256, 64, 256, 1, 1),
    ("l2.c1", 64, 256, 256, 256, 128, 1, 1),
    ("l3.c2", 16, 64, 64, 256, 256, 3, 1),
    ("mb.proj", 32, 64, 64, 672, 112, 1, 1),
    ("mb.exp", 32, 64, 64, 112, 672, 1, 1),
    ("b3.exp", 32, 256, 256, 24, 72, 1, 1),
]


def main():
    out, ref = sys.argv[1], "--ref" in sys.argv
    dev = torch.device("cuda")
    res = {}
    for name, B, H, W, cin, cout, k, s in SHAPES:
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(B, H, W, cin, device=dev, generator=g)
        OH, OW = (H + 2 * (k // 2) - k) // s + 1, (W + 2 * (k // 2) - k) // s + 1
        dy = torch.randn(B, OH, OW, cout, device=dev, generator=g)
        w = torch.empty(cout, cin, k, k, device=dev)
        dw = T._wgrad(x, dy, w, s, k // 2)
        torch.cuda.synchronize()
        res[name] = dw.cpu()
        msg = f"{name:8s} finite={bool(torch.isfinite(dw).all())}"
        if ref and k == 1:
            xm, dm = x.reshape(-1, cin), dy.reshape(-1, cout)
            acc = torch.zeros(cin, cout, dtype=torch.float64, device=dev)
            for i in range(0, xm.shape[0], 1 << 20):
                acc += (xm[i:i + (1 << 20)].t() @ dm[i:i + (1 << 20)]).double()
            r = acc.t().reshape(cout, cin, 1, 1)
            msg += " rel_err_vs_mm %.2e" % float((dw.double() - r).abs().max() / r.abs().max())
        print(msg, flush=True)
        del x, dy
        torch.cuda.empty_cache()
    torch.save(res, out)


if __name__ == "__main__":
    main()
