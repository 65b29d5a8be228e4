"""Time the R50 7x7/s2 stem (forward + weight gradient) at the C3 shape.

  python3 tools/stem7_bench.py [--batch 64 --size 1024]
JABD_STEM7=0 in the environment selects the generic kernels (A/B).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]
import torch  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from jabd_amd import train as T
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(a.batch, 3, a.size, a.size, device=dev, generator=g)
    w = torch.nn.Parameter(torch.randn(64, 3, 7, 7, device=dev, generator=g) / 147 ** 0.5)
    y = T.ConvFn.apply(x, w, None, 2, 3, True)
    dy = torch.randn(y.shape, device=dev, generator=g)
    OH = y.shape[1]
    flop = 2.0 * a.batch * OH * OH * 147 * 64
    fwd = timed(lambda: T.ConvFn.apply(x, w, None, 2, 3, True), a.iters)

    def bwd():
        w.grad = None
        T._wgrad(x, dy, w, 2, 3, True)
    wg = timed(bwd, a.iters)
    out = {"stem7": os.environ.get("JABD_STEM7", "1"), "batch": a.batch, "size": a.size,
           "fwd_ms": fwd, "fwd_tflops": flop / fwd / 1e9, "wgrad_ms": wg, "wgrad_tflops": flop / wg / 1e9,
           "fwd_frac": flop / fwd / 1e9 / 157.3, "wgrad_frac": flop / wg / 1e9 / 157.3}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
