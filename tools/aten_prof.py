"""Attribute the ATen fills / copies of a training step, including the ones
the autograd engine issues on its backward thread (torch.profiler, which
records every thread; TorchDispatchMode in aten_trace.py sees only the
forward).  Prints, per (op, enclosing autograd node or Python frame), the
number of calls in one step.

  python3 tools/aten_prof.py [--kind mnv3] [--batch 8] [--size 512]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from jabd_amd import optim, parallel, synth  # noqa: E402
from nets.retinaface_training import MultiBoxLoss  # noqa: E402
from utils.anchors import Anchors  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--kind", default="mnv3")
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--size", type=int, default=512)
a = ap.parse_args()
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
WATCH = ("aten::fill_", "aten::zero_", "aten::copy_", "aten::add", "aten::add_", "aten::cat",
         "aten::clone", "aten::sum", "aten::index_put_", "aten::index", "aten::mul",
         "aten::_foreach_add_", "aten::to", "aten::_to_copy")
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
    parallel.train_step(model, crit, opt, x, tg, pri)
    torch.cuda.synchronize()
evs = prof.events()
byid = {e.id: e for e in evs}
agg = collections.Counter()
for e in evs:
    if e.name not in WATCH:
        continue
    # nearest enclosing non-aten op (autograd node, Python function) as the site
    p = e.cpu_parent
    chain = []
    while p is not None and len(chain) < 3:
        if not p.name.startswith("aten::"):
            chain.append(p.name.split("(")[0][:60])
        p = p.cpu_parent
    st = [s for s in (e.stack or []) if "jabd_amd" in s or "/nets/" in s or "parallel" in s]
    site = " <- ".join(chain) if chain else "-"
    if st:
        site += " | " + st[0].split("/")[-1][:60]
    agg[(e.name, site)] += 1
for (n, site), c in agg.most_common(60):
    print(f"{c:5d}  {n:18s} {site}")
