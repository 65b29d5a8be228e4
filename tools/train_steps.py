"""Run a few JABD training steps (for rocprofv3 --kernel-trace --stats).

  python3 tools/train_steps.py --kind mnv3|beca|small|r50 [--batch 32] [--steps 3]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]
import torch  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--kind", default="mnv3")
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--size", type=int, default=1024)
ap.add_argument("--steps", type=int, default=3)
a = ap.parse_args()
r = bench.train_bench(a.kind, a.batch, a.size, a.steps, 1, torch.device("cuda"), None, 0)
print(r)
