"""Stage-by-stage check of the graphed bs1 predict path (diagnostics).

  python3 tools/graph_check.py [--kind mnv3] [--size 640] [--no-detect]
Prints one line per stage; a faulthandler traceback after --limit seconds.
"""
import argparse
import faulthandler
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]


def say(*a):
    print(f"[{time.perf_counter() - T0:7.2f}s]", *a, flush=True)


T0 = time.perf_counter()
ap = argparse.ArgumentParser()
ap.add_argument("--kind", default="mnv3")
ap.add_argument("--size", type=int, default=640)
ap.add_argument("--no-detect", action="store_true")
ap.add_argument("--no-splitk", action="store_true")
ap.add_argument("--limit", type=int, default=90)
ap.add_argument("--zeros", action="store_true", help="eager detect on an all-zero input first")
ap.add_argument("--test-seq", action="store_true", help="tests/test_prep.py's graphed sequence")
ap.add_argument("--sync", action="store_true", help="(--test-seq) synchronise between the stages")
ap.add_argument("--between", default="", help="fwd|det|both: eager work between graph replays")
a = ap.parse_args()
faulthandler.dump_traceback_later(a.limit, exit=True)
import torch  # noqa: E402
import bench  # noqa: E402
from jabd_amd import functional as F  # noqa: E402
from jabd_amd import ops  # noqa: E402
from utils.anchors import Anchors  # noqa: E402
dev = torch.device("cuda")
net, cfg = bench._weights_init_model(a.kind)
net = net.eval().to(dev)
pri = Anchors(cfg, image_size=(a.size, a.size)).get_anchors().to(dev).float()
var = cfg["variance"]
x = (torch.rand(1, 3, a.size, a.size, generator=torch.Generator().manual_seed(1)) * 255 - 117).to(dev)
sk = F.split_k() if not a.no_splitk else torch.no_grad()


def body():
    with torch.no_grad(), (F.split_k() if not a.no_splitk else torch.no_grad()):
        out = net(x)
        if a.no_detect:
            return out
        return ops.detect(*out, pri, var, 0.5, 0.3)


say("model ready")
if a.between:
    from jabd_amd.predict import graphed_detect
    with torch.no_grad():
        out = net(x)
        rows, nk = graphed_detect(net, x, pri, var, 0.5, 0.3)
        torch.cuda.synchronize()
        say("graph built, n_keep", int(nk[0]))
        for it in range(3):
            if a.between in ("fwd", "both"):
                with F.split_k():
                    out = net(x)
                torch.cuda.synchronize()
                say(it, "eager forward done")
            if a.between in ("det", "both"):
                r0, n0 = ops.detect(*out, pri, var, 0.5, 0.3)
                torch.cuda.synchronize()
                say(it, "eager detect done", int(n0[0]))
            rows, nk = graphed_detect(net, x, pri, var, 0.5, 0.3)
            torch.cuda.synchronize()
            say(it, "replay done", int(nk[0]))
    faulthandler.cancel_dump_traceback_later()
    sys.exit(0)
if a.test_seq:
    from jabd_amd.predict import graphed_detect
    g = torch.Generator().manual_seed(a.size)
    for it in range(2):
        x = (torch.rand(1, 3, a.size, a.size, generator=g) * 255 - 117).to(dev)
        with torch.no_grad():
            with F.split_k():
                out = net(x)
            if a.sync:
                torch.cuda.synchronize()
                say(it, "eager forward done")
            r0, n0 = ops.detect(*out, pri, var, 0.5, 0.3)
            if a.sync:
                torch.cuda.synchronize()
                say(it, "eager detect done", int(n0[0]))
            r1, n1 = graphed_detect(net, x, pri, var, 0.5, 0.3)
            say(it, "graphed_detect returned")
            if a.sync:
                torch.cuda.synchronize()
                say(it, "graphed detect done", int(n1[0]))
        say(it, "n_keep", int(n0[0]), int(n1[0]))
    faulthandler.cancel_dump_traceback_later()
    sys.exit(0)
if a.zeros:
    x0 = torch.zeros_like(x)
    for i in range(3):
        with torch.no_grad(), F.split_k():
            o0 = net(x0)
        torch.cuda.synchronize()
        say("zeros forward done")
        r0 = ops.detect(*o0, pri, var, 0.5, 0.3)
        torch.cuda.synchronize()
        say("zeros detect done, n_keep", int(r0[1][0]), "scores>0.5:", int((o0[1][0, :, 1] > 0.5).sum()))
r = body()
torch.cuda.synchronize()
say("eager done")
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for _ in range(2):
        body()
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
say("side-stream warmup done")
g = torch.cuda.CUDAGraph()
say("capture begin")
with torch.cuda.graph(g):
    out = body()
say("capture end")
g.replay()
say("replay issued")
torch.cuda.synchronize()
say("replay done")
if not a.no_detect:
    say("n_keep eager", int(r[1][0]), "graph", int(out[1][0]))
t0 = time.perf_counter()
for _ in range(50):
    g.replay()
torch.cuda.synchronize()
say(f"graph replay {(time.perf_counter() - t0) / 50 * 1e3:.3f} ms/iter")
faulthandler.cancel_dump_traceback_later()
