"""Prior boxes — drop-in for the reference utils/anchors.py:8-42.

Priors are generated once per (cfg, image size) on the host in double
precision (exactly the reference's arithmetic and emission order: level ->
row -> column -> min_size), converted to fp32 once, and cached; there is no
per-step host work.  (The reference module's import-time print of 29518 is
not reproduced.)
"""
import itertools
from math import ceil

import numpy as np
import torch

_CACHE = {}


class Anchors(object):
    def __init__(self, cfg, image_size=None):
        self.min_sizes = cfg["min_sizes"]
        self.steps = cfg["steps"]
        self.clip = cfg["clip"]
        self.image_size = image_size
        self.feature_maps = [[ceil(self.image_size[0] / s), ceil(self.image_size[1] / s)]
                             for s in self.steps]

    def get_anchors(self):
        key = (tuple(map(tuple, self.min_sizes)), tuple(self.steps), bool(self.clip),
               tuple(self.image_size))
        hit = _CACHE.get(key)
        if hit is None:
            H, W = self.image_size[0], self.image_size[1]
            rows = []
            for k, (fh, fw) in enumerate(self.feature_maps):
                st = self.steps[k]
                for i, j in itertools.product(range(fh), range(fw)):
                    for m in self.min_sizes[k]:
                        rows.append(((j + 0.5) * st / W, (i + 0.5) * st / H, m / W, m / H))
            hit = torch.from_numpy(np.asarray(rows, dtype=np.float64).reshape(-1, 4)
                                   .astype(np.float32))
            if self.clip:
                hit.clamp_(max=1, min=0)
            _CACHE[key] = hit
        return hit.clone()
