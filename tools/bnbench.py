"""BatchNorm training kernels at the C4 (MobileNetV3, bs32 1024²) shapes:
HIP-event time and algorithmic HBM bandwidth of the statistics pass, the
normalise+activation pass and the backward (partials + apply).

  python3 tools/bnbench.py [--reps 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]
import torch  # noqa: E402

from jabd_amd import train as T  # noqa: E402

# (name, rows M = B*H*W, channels C)
SHAPES = [("b2.bn1 512²x64", 32 * 512 * 512, 64), ("b1.bn 512²x16", 32 * 512 * 512, 16),
          ("b3.bn1 256²x72", 32 * 256 * 256, 72), ("b5.bn1 128²x120", 32 * 128 * 128, 120),
          ("b12.bn1 64²x672", 32 * 64 * 64, 672), ("b15.bn1 32²x960", 32 * 32 * 32, 960),
          ("ssh 128²x12", 32 * 128 * 128, 12)]


def timed(fn, reps):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    for name, M, C in SHAPES:
        x = torch.randn((M // 1024, 32, 32, C), device=dev)
        bn = torch.nn.BatchNorm2d(C).to(dev)
        x.requires_grad_(True)
        fwd = lambda: T.BnActFn.apply(x, bn.weight, bn.bias, None, bn.running_mean,  # noqa: E731
                                      bn.running_var, "relu", 0.0, 0.1, 1e-5)
        y = fwd()
        dy = torch.randn_like(y)
        t_f = timed(lambda: fwd(), a.reps)
        t_fb = timed(lambda: torch.autograd.grad(fwd(), (x, bn.weight, bn.bias), dy), a.reps)
        nb = 4.0 * M * C
        # forward: stats read + apply read/write = 3 passes; backward: part
        # (x, dy) + apply (x, dy, dx) = 5 passes
        print("%-18s fwd %8.1f us %6.0f GB/s | bwd %8.1f us %6.0f GB/s" % (
            name, t_f, 3 * nb / t_f / 1e3, t_fb - t_f, 5 * nb / (t_fb - t_f) / 1e3), flush=True)


if __name__ == "__main__":
    main()
