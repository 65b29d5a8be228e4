"""List every ATen op of one training step that runs a GPU kernel, with the
Python line that issued it, forward and backward alike: autograd runs the
backward on the calling thread (set_multithreading_enabled(False)), so one
TorchDispatchMode sees both passes.

  python3 tools/aten_sites.py [--kind mnv3] [--batch 8] [--size 512]
"""
import argparse
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

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

# ops that only make views / metadata or allocate without writing
QUIET = {"empty", "empty_strided", "empty_like", "view", "_unsafe_view", "reshape", "permute",
         "as_strided", "t", "transpose", "expand", "slice", "select", "unsqueeze", "squeeze",
         "detach", "alias", "lift_fresh", "_to_copy_noop", "resize_", "set_", "split",
         "unbind", "narrow", "contiguous", "is_same_size", "_local_scalar_dense", "item",
         "clamp_min", "_reshape_alias", "unfold", "diagonal", "view_as", "squeeze_"}
sites = collections.Counter()


class Mode(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        out = func(*args, **kwargs)
        name = func.__name__.split(".")[0]
        if name in QUIET:
            return out
        tens = [t for t in list(args) + list(kwargs.values()) + [out]
                if isinstance(t, torch.Tensor)]
        if not any(t.is_cuda for t in tens):
            return out
        st = [f for f in traceback.extract_stack()[:-1]
              if ("jabd_amd" in f.filename or "/nets/" in f.filename or "/utils/" in f.filename)
              and "_python_dispatch" not in f.filename]
        site = "%s:%d %s" % (os.path.basename(st[-1].filename), st[-1].lineno, st[-1].name) \
            if st else "?"
        node = torch._C._current_autograd_node()
        if node is not None:
            site += " [%s]" % node.name()
        elif name in ("add", "add_"):
            shp = [tuple(t.shape) for t in tens[:1]]
            site += " %s" % shp
        sites[(name, site)] += 1
        return out


torch.autograd.set_multithreading_enabled(False)
with Mode():
    parallel.train_step(model, crit, opt, x, tg, pri)
torch.cuda.synchronize()
print("total", sum(sites.values()))
for (n, s), c in sites.most_common():
    print(f"{c:5d}  {n:24s} {s}")
