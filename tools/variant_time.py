"""Eval-forward time of the detector variants at the C2 shape (bs32 1024^2).

  python3 tools/variant_time.py [--kinds beca,small,mnv3] [--steps 5]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]
import torch  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--kinds", default="beca,small,mnv3")
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--size", type=int, default=1024)
a = ap.parse_args()
for k in a.kinds.split(","):
    print(json.dumps(bench.variant_forward(k, torch.device("cuda"), a.size, a.batch, a.steps)),
          flush=True)
