"""Attribute the ATen ops (fills, copies, adds, cats) of a training step to
the Python lines that issue them (torch.profiler with stacks).

  python3 tools/aten_trace.py [--kind mnv3] [--batch 8] [--size 512]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--kind", default="mnv3")
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--size", type=int, default=512)
a = ap.parse_args()

from jabd_amd import optim, parallel, synth  # noqa: E402
from nets.retinaface_training import MultiBoxLoss  # noqa: E402
from utils.anchors import Anchors  # noqa: E402

dev = torch.device("cuda")
RetinaFace, cfg = bench.detector(a.kind)
model = RetinaFace(cfg=cfg, mode="train").to(dev).train()
opt = optim.Adam(model.parameters(), 1e-3, weight_decay=5e-4)
crit = MultiBoxLoss(2, 0.35, 7, cfg["variance"], True)
pri = Anchors(cfg, image_size=(a.size, a.size)).get_anchors().to(dev)
x = synth.images(a.batch, a.size, seed=1, device=dev)
tg = [torch.from_numpy(t).to(dev) for t in synth.targets(a.batch, a.size, seed=2)]
for _ in range(2):
    parallel.train_step(model, crit, opt, x, tg, pri)
torch.cuda.synchronize()
WATCH = {"fill_", "zero_", "copy_", "add_", "add", "cat", "zeros", "clone", "mul", "sum", "div",
         "new_zeros", "new_ones", "ones", "empty_like"}
import traceback  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

agg = collections.Counter()


class Watch(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.__name__.split(".")[0]
        if name in WATCH:
            fr = [f for f in traceback.extract_stack()[:-1]
                  if ("jabd_amd" in f.filename or "/nets/" in f.filename)]
            where = (" <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}"
                                 for f in reversed(fr[-3:])) if fr else "<autograd/c++>")
            agg[(name, where)] += 1
        return func(*args, **(kwargs or {}))


with Watch():
    parallel.train_step(model, crit, opt, x, tg, pri)
torch.cuda.synchronize()
for (name, where), n in agg.most_common(80):
    print(f"{n:5d}  {name:10s} {where}")
