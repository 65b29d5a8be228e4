"""A/B of the streaming 1x1 GEMM form (conv1x1_m32s_kernel) against
conv1x1_m32_kernel: run under JABD_M32S=1 and JABD_M32S=0 with the same
--out prefix, then --compare.  Every output (plain / bias+act / residual
data gradient, statistics rows -> mean / invstd, BatchNorm-backward sums ->
dx / dgamma / dbeta) must be bit-identical; also prints per-shape times.

  python tools/m32s_ab.py --out gpurun_out/m32s_on      (JABD_M32S=1)
  python tools/m32s_ab.py --out gpurun_out/m32s_off     (JABD_M32S=0)
  python tools/m32s_ab.py --compare gpurun_out/m32s_on gpurun_out/m32s_off
"""
import argparse
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]

# (name, B, H, W, cin, cout) 1x1 stride-1 GEMMs with K = cin
SHAPES = [
    ("k64n256", 2, 40, 36, 64, 256), ("k64n64", 3, 17, 19, 64, 64),
    ("k128n512", 2, 21, 18, 128, 512), ("k64n96", 1, 9, 7, 64, 96),
    ("k128n128", 2, 33, 31, 128, 128), ("k64n32", 1, 5, 3, 64, 32),
    ("l1c3", 16, 256, 256, 64, 256), ("l2c3", 16, 128, 128, 128, 512),
]


def run(out):
    from jabd_amd import train as T
    dev = torch.device("cuda")
    res = {}
    for name, B, H, W, cin, cout in SHAPES:
        g = torch.Generator().manual_seed(cin * 131 + cout)
        x = ((torch.randn(B, H, W, cin, generator=g) + 1.0) * 3.0).to(dev)
        w = (torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5).to(dev)
        b = torch.randn(cout, generator=g).to(dev)
        r = torch.randn(B, H, W, cout, generator=g).to(dev)
        bn = torch.nn.BatchNorm2d(cout).to(dev)
        res[name + ".plain"] = T._conv_fwd(x, w, b, 1, 0)
        y, st = T._conv_fwd_stats(x, w, bn, 1, 0)
        res[name + ".st_y"] = y
        if st is not None:
            res[name + ".st_mean"], res[name + ".st_invstd"] = st
        # data gradient of a conv cout -> cin (K = cin here) with the residual
        wt = w.reshape(cout, cin).t().contiguous().reshape(cin, cout, 1, 1)
        dy = torch.randn(B, H, W, cin, generator=g).to(dev)
        res[name + ".dres"] = T._dgrad_1x1_res(dy, wt, r)
        # BatchNorm-backward sums form: the data gradient is the dy of a BN over cout channels
        xb = ((torch.randn(B, H, W, cout, generator=g) + 2.0)).to(dev)
        xm = xb.reshape(-1, cout).double()
        stb = ((1 + 0.3 * torch.randn(cout, generator=g)).to(dev),
               (0.2 * torch.randn(cout, generator=g)).to(dev),
               xm.mean(0).float(), (xm.var(0, unbiased=False) + 1e-5).rsqrt().float())
        d1, part = T._dgrad_bn_sums(dy, wt, 1, 0, H, W, xb, stb, "relu")
        res[name + ".bb_d"] = d1
        if part is not None:
            dx, dgm, dbt, _ = T._bn_bwd_rows(d1, xb, stb, "relu", part)
            res[name + ".bb_dx"], res[name + ".bb_dg"], res[name + ".bb_db"] = dx, dgm, dbt
        torch.cuda.synchronize()
        # timing of the plain forward and the statistics form
        for tag, fn in (("plain", lambda: T._conv_fwd(x, w, None, 1, 0)),
                        ("stats", lambda: T._conv_fwd_stats(x, w, bn, 1, 0))):
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            torch.cuda.synchronize()
            print("%-9s %-5s M %8d K %4d N %4d  %9.1f us" % (name, tag, B * H * W, cin, cout,
                                                             e0.elapsed_time(e1) * 100.0),
                  flush=True)
    import hashlib
    import json
    digest = {k: [hashlib.sha256(v.detach().contiguous().cpu().numpy().tobytes()).hexdigest(),
                  float(v.double().sum())] for k, v in res.items()}
    with open(out + ".json", "w") as f:
        json.dump(digest, f, indent=1, sort_keys=True)
    print("saved", len(res), "digests to", out + ".json")


def compare(a, b):
    import json
    ta, tb = (json.load(open(p + ".json")) for p in (a, b))
    bad = 0
    for k in sorted(ta):
        if k not in tb or ta[k][0] != tb[k][0]:
            bad += 1
            print("DIFF", k, ta[k][1], tb[k][1] if k in tb else None)
    print("compared %d tensors, %d differ" % (len(ta), bad))
    return bad


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    ap.add_argument("--compare", nargs=2)
    args = ap.parse_args()
    if args.compare:
        sys.exit(1 if compare(*args.compare) else 0)
    run(args.out)
