"""bs1 predict.py get_FPS loop (bench.predict_fps) for one detector / size, for
rocprofv3 --kernel-trace --stats and per-stage host timing.

  python3 tools/predict_steps.py --kind r50 --size 640 --iters 50
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--kind", default="r50")
ap.add_argument("--size", type=int, default=640)
ap.add_argument("--iters", type=int, default=50)
a = ap.parse_args()
from jabd_amd import ops  # noqa: E402
from utils.anchors import Anchors  # noqa: E402
dev = torch.device("cuda")
net, cfg = bench._weights_init_model(a.kind)
net = net.eval().to(dev)
img = np.random.default_rng(a.size).integers(0, 256, (a.size * 3 // 4, a.size, 3)).astype(np.float32)
x = ops.letterbox(torch.from_numpy(img).to(dev), (a.size, a.size), mean=(104.0, 117.0, 123.0))
pri = Anchors(cfg, image_size=(a.size, a.size)).get_anchors().to(dev).float()
var = cfg["variance"]
for _ in range(5):
    with torch.no_grad():
        rows, nk = ops.detect(*net(x), pri, var, 0.5, 0.3)
torch.cuda.synchronize()
tf = td = 0.0
for _ in range(a.iters):
    t0 = time.perf_counter()
    with torch.no_grad():
        out = net(x)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        rows, nk = ops.detect(*out, pri, var, 0.5, 0.3)
        k = int(nk[0])
        rows[0, :k].cpu()
    t2 = time.perf_counter()
    tf += t1 - t0
    td += t2 - t1
print(f"{a.kind} {a.size}: forward {tf / a.iters * 1e3:.2f} ms, detect+copy {td / a.iters * 1e3:.2f} ms, "
      f"kept {k}")
