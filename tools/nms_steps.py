"""C5 NMS runs for rocprofv3 --kernel-trace --stats (bench.nms_bench: 8 images
x 100k clustered boxes, iou 0.3, one warm-up + `reps` timed batched calls).

  python3 tools/nms_steps.py [--reps 5]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]
import torch  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
print(bench.nms_bench(torch.device("cuda"), reps=a.reps))
