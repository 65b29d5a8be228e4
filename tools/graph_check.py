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
