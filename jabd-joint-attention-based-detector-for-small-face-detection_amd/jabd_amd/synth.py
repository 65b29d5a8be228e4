"""Synthetic WIDER-FACE-shaped inputs — no dataset ships here.

Images: uniform [0,255) minus the BGR means (utils/utils.py:28-30), NCHW.
Targets: per image n ~ clip(round(LogNormal(ln 8, 1)), 1, 1000) faces, the
15-column layout of utils/dataloader.py:33-58,145-147 (x1,y1,x2,y2, five
landmark points, label +1 / -1 with zeroed landmarks), normalised coords.
NMS sweep (C5): clustered boxes with injected exact score ties.
"""
import numpy as np
import torch

BGR_MEAN = (104.0, 117.0, 123.0)


def images(batch, size, seed=1234, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand((batch, 3, size, size), generator=g) * 255.0
    x -= torch.tensor(BGR_MEAN).view(1, 3, 1, 1)
    return x.to(device)


def targets(batch, size, seed=4321, max_faces=1000):
    """List of B float32 numpy arrays [n_i, 15]."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(batch):
        n = int(np.clip(np.round(rng.lognormal(np.log(8.0), 1.0)), 1, max_faces))
        side = np.exp(rng.uniform(np.log(4.0), np.log(512.0), n)) / size
        ar = rng.uniform(0.7, 1.4, n)
        w = np.minimum(side, 0.999)
        h = np.minimum(side * ar, 0.999)
        cx = rng.uniform(w / 2, 1 - w / 2)
        cy = rng.uniform(h / 2, 1 - h / 2)
        t = np.zeros((n, 15), dtype=np.float64)
        t[:, 0], t[:, 1] = cx - w / 2, cy - h / 2
        t[:, 2], t[:, 3] = cx + w / 2, cy + h / 2
        for k in range(5):
            t[:, 4 + 2 * k] = rng.uniform(t[:, 0], t[:, 2])
            t[:, 5 + 2 * k] = rng.uniform(t[:, 1], t[:, 3])
        neg = rng.uniform(size=n) < 0.2
        t[:, 14] = np.where(neg, -1.0, 1.0)
        t[neg, 4:14] = 0.0
        out.append(t.astype(np.float32))
    return out


def nms_boxes(batch, n, seed=99, centres=500, tie_frac=0.02):
    """C5 sweep: boxes [B,n,4], scores [B,n] (float32 numpy)."""
    rng = np.random.default_rng(seed)
    boxes = np.empty((batch, n, 4), np.float32)
    scores = np.empty((batch, n), np.float32)
    for b in range(batch):
        c = rng.uniform(0, 1, (centres, 2))
        pick = rng.integers(0, centres, n)
        ctr = c[pick] + rng.normal(0, 0.01, (n, 2))
        wh = np.exp(rng.uniform(np.log(2 / 2048), np.log(0.25), (n, 2)))
        boxes[b, :, :2] = ctr - wh / 2
        boxes[b, :, 2:] = ctr + wh / 2
        s = rng.uniform(0.5, 1.0, n).astype(np.float32)
        tie = rng.uniform(size=n) < tie_frac
        src = rng.integers(0, n, n)
        s[tie] = s[src[tie]]
        scores[b] = s
    return boxes, scores
